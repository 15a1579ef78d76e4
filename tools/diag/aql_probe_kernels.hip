// Kernels of aql_probe.cpp (tools/diag), built as a bare gfx950 code object:
//   hipcc --offload-arch=gfx950 --cuda-device-only --no-gpu-bundle-output -O3 -o aql_probe_kernels.co aql_probe_kernels.hip
#include <hip/hip_runtime.h>
typedef float v4f __attribute__((ext_vector_type(4)));
extern "C" __global__ __launch_bounds__(64) void k_empty() {}
extern "C" __global__ __launch_bounds__(64) void k_copy(const v4f *in, v4f *out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    v4f v = in[i];
    v[0] += 1.f;
    __builtin_nontemporal_store(v, out + i);
}

// Coherence probe (aql_probe.cpp, mode "coherence"): k_write stores seq into every word with a plain store
// (pol 0) or a nontemporal one (pol 1); k_check reads every word through a permuted workgroup -> block
// mapping (so blocks move between XCDs and CUs from one dispatch to the next) and counts the words that are not
// `want` (a reader that sees a stale copy).
extern "C" __global__ __launch_bounds__(64) void k_write(unsigned *buf, unsigned seq, int pol) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    if (pol)
        __builtin_nontemporal_store(seq, buf + i);
    else
        buf[i] = seq;
}
extern "C" __global__ __launch_bounds__(64) void k_check(const unsigned *buf, unsigned want, unsigned mul,
                                                         unsigned add, unsigned long long *errors, unsigned nblk) {
    const unsigned blk = (blockIdx.x * mul + add) % nblk;
    const unsigned v = buf[blk * 64 + threadIdx.x];
    if (v != want) __hip_atomic_fetch_add(errors, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
