// kernarg_probe.hip's kernels, compiled with -mllvm -amdgpu-kernarg-preload-count=16 (tools/diag/Makefile).
#include "kernarg_probe.h"

__global__ __launch_bounds__(64) void k_copy_pre(const v4f *in, v4f *out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    v4f v = in[i];
    v[0] += 1.f;
    __builtin_nontemporal_store(v, out + i);
}

__global__ __launch_bounds__(64) void k_copy_big_pre(BigArgs a) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    v4f v = a.in[i];
    v[0] += a.pad[3];
    __builtin_nontemporal_store(v, a.out + i);
}

void launch_copy_preload(hipStream_t st, v4f *in, v4f *out) {
    hipLaunchKernelGGL(k_copy_pre, dim3(kBlocks), dim3(64), 0, st, in, out);
}
void launch_copy_big_preload(hipStream_t st, v4f *in, v4f *out) {
    BigArgs a{};
    a.in = in;
    a.out = out;
    hipLaunchKernelGGL(k_copy_big_pre, dim3(kBlocks), dim3(64), 0, st, a);
}
