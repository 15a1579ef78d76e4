// Does the kernel-argument fetch sit on the step's critical path?  The same small kernel (2,048 one-wavefront
// workgroups, the headline step's grid: each lane loads 16 B and stores 16 B) built twice: here as usual (its
// pointers arrive by s_load from the kernarg segment) and in kernarg_probe_pre.hip with
// -mllvm -amdgpu-kernarg-preload-count=16 (the pointers preloaded into SGPRs at wave launch where the firmware
// supports it).  Each kernel runs as 24 dependent launches captured in a hipGraph (a day's steps); the time per
// node is the replay's HIP-event time / 24.  A third kernel carries a 600 B argument block (the step's size) and
// reads one field behind it, a fourth does nothing; and the empty kernel's node time against its grid.
// Build: make -C tools/diag kernarg_probe      Run: tools/diag/kernarg_probe [replays]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernarg_probe.h"

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

__global__ __launch_bounds__(64) void k_empty() {}
__global__ __launch_bounds__(1024) void k_empty_any() {}

__global__ __launch_bounds__(64) void k_copy(const v4f *in, v4f *out) {
    const int i = blockIdx.x * 64 + threadIdx.x;
    v4f v = in[i];
    v[0] += 1.f;
    __builtin_nontemporal_store(v, out + i);
}

__global__ __launch_bounds__(64) void k_copy_big(BigArgs a) {   // the pointers behind 600 B of arguments
    const int i = blockIdx.x * 64 + threadIdx.x;
    v4f v = a.in[i];
    v[0] += a.pad[3];
    __builtin_nontemporal_store(v, a.out + i);
}

static double per_node_us(hipStream_t st, void (*launch)(hipStream_t, v4f *, v4f *), v4f *in, v4f *out,
                          int replays) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int t = 0; t < 24; ++t) launch(st, t & 1 ? out : in, t & 1 ? in : out);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<double> us;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a, st));
        for (int i = 0; i < replays; ++i) CK(hipGraphLaunch(ge, st));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, a, b));
        us.push_back(ms * 1e3 / (24.0 * replays));
    }
    std::sort(us.begin(), us.end());
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return us[us.size() / 2];
}

static void l_empty(hipStream_t st, v4f *, v4f *) { hipLaunchKernelGGL(k_empty, dim3(kBlocks), dim3(64), 0, st); }
static int g_blocks = kBlocks, g_threads = 64;
static void l_empty_grid(hipStream_t st, v4f *, v4f *) {
    hipLaunchKernelGGL(k_empty_any, dim3(g_blocks), dim3(g_threads), 0, st);
}
static void l_copy(hipStream_t st, v4f *in, v4f *out) {
    hipLaunchKernelGGL(k_copy, dim3(kBlocks), dim3(64), 0, st, in, out);
}
static void l_copy_big(hipStream_t st, v4f *in, v4f *out) {
    BigArgs a{};
    a.in = in;
    a.out = out;
    hipLaunchKernelGGL(k_copy_big, dim3(kBlocks), dim3(64), 0, st, a);
}

int main(int argc, char **argv) {
    const int replays = argc > 1 ? std::atoi(argv[1]) : 200;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    v4f *in, *out;
    CK(hipMalloc(&in, sizeof(v4f) * kBlocks * 64));
    CK(hipMalloc(&out, sizeof(v4f) * kBlocks * 64));
    CK(hipMemset(in, 0, sizeof(v4f) * kBlocks * 64));
    struct Row {
        const char *name;
        void (*launch)(hipStream_t, v4f *, v4f *);
    } rows[] = {{"empty", l_empty},
                {"copy", l_copy},
                {"copy_preload", launch_copy_preload},
                {"copy_big_args", l_copy_big},
                {"copy_big_args_preload", launch_copy_big_preload}};
    // the empty kernel's node time against its grid: workgroups x threads per workgroup
    for (int threads : {64, 256}) {
        for (int blocks : {1, 256, 1024, 2048, 4096, 8192}) {
            g_blocks = blocks;
            g_threads = threads;
            std::printf("grid  empty  %5d x %4d  %.3f us per graph node\n", blocks, threads,
                        per_node_us(st, l_empty_grid, in, out, replays));
        }
    }
    for (int pass = 0; pass < 2; ++pass)
        for (const Row &r : rows)
            std::printf("pass %d  %-22s %.3f us per graph node\n", pass, r.name, per_node_us(st, r.launch, in, out, replays));
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
