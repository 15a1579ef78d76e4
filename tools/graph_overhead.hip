// graph_overhead.hip -- what a dependent kernel boundary costs (not part of the product).
//   hipcc --offload-arch=gfx950 -O3 -o tools/graph_overhead tools/graph_overhead.hip && tools/graph_overhead
//
// The bench replays days as hipGraphs: 25 dependent kernels per day, each step kernel 2,048 one-wavefront
// workgroups.  Here, at that grid, the mean time per kernel of
//   empty    a kernel that does nothing
//   store    each lane stores 16 B (2 MB per launch)
//   copy     the step's bytes as a float4 copy (11.0 MB read, 14.5 MB written per launch: 1,557,504 threads)
// launched (a) back to back on one stream and (b) as a captured graph of the same 480 launches.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void k_empty(float *) {}
__global__ __launch_bounds__(1024) void k_empty_wide(float *) {}
__global__ __launch_bounds__(64) void k_store(v4f *out) {
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    __builtin_nontemporal_store(v4f{1.f, 2.f, 3.f, 4.f}, out + i);
}
__global__ __launch_bounds__(256) void k_copy(const v4f *__restrict__ in, v4f *__restrict__ out, long nr, long nw) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    v4f v = {0.f, 0.f, 0.f, 0.f};
    if (i < nr) v = in[i];
    if (i < nw) __builtin_nontemporal_store(v, out + i);
}

template <class F>
void measure(const char *name, F launch) {
    constexpr int N = 480, R = 10;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < N; ++i) launch(s);   // warm
    CK(hipStreamSynchronize(s));
    float best_stream = 1e30f;
    for (int r = 0; r < R; ++r) {
        CK(hipEventRecord(a, s));
        for (int i = 0; i < N; ++i) launch(s);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best_stream = ms < best_stream ? ms : best_stream;
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < N; ++i) launch(s);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best_graph = 1e30f;
    for (int r = 0; r < R; ++r) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        best_graph = ms < best_graph ? ms : best_graph;
    }
    printf("%-10s stream back to back %7.3f us/kernel   graph %7.3f us/kernel\n", name, best_stream * 1e3f / N,
           best_graph * 1e3f / N);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(s));
}

int main() {
    const long nr = 11010048 / 16, nw = 14483456 / 16, n = nr > nw ? nr : nw;
    v4f *in, *out;
    CK(hipMalloc(&in, nr * 16));
    CK(hipMalloc(&out, n * 16));
    CK(hipMemset(in, 0, nr * 16));
    // the boundary's fixed part against its per-workgroup part: empty kernels of other grids
    const int grids[][2] = {{1, 64}, {256, 64}, {512, 64}, {1024, 64}, {4096, 64}, {512, 256}, {256, 512}, {2048, 256}};
    for (const auto &g : grids) {
        char name[32];
        snprintf(name, sizeof name, "empty%dx%d", g[0], g[1]);
        measure(name, [&](hipStream_t s) {
            if (g[1] == 64)
                hipLaunchKernelGGL(k_empty, dim3(g[0]), dim3(g[1]), 0, s, (float *)out);
            else
                hipLaunchKernelGGL(k_empty_wide, dim3(g[0]), dim3(g[1]), 0, s, (float *)out);
        });
    }
    for (int rep = 0; rep < 2; ++rep) {
        measure("empty", [&](hipStream_t s) { hipLaunchKernelGGL(k_empty, dim3(2048), dim3(64), 0, s, (float *)out); });
        measure("store", [&](hipStream_t s) { hipLaunchKernelGGL(k_store, dim3(2048), dim3(64), 0, s, out); });
        measure("copy", [&](hipStream_t s) {
            hipLaunchKernelGGL(k_copy, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, nr, nw);
        });
    }
    CK(hipFree(in));
    CK(hipFree(out));
    return 0;
}
