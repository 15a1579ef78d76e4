// membench.hip -- memory-pattern microbenchmarks behind the step/reset kernel layout choices.
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -o membench tools/membench.hip
//
//   copy      : float4 stream, R bytes read + W bytes written (the bandwidth floor of a step)
//   store_f64 : dense f64 stores, one per lane               (reset: dense aux timeline)
//   store_msk : f64 stores with ~p of lanes active           (masked partial-line stores)
//   load_msk  : f64 loads with ~p of lanes active
// Each case: 200 back-to-back launches timed with events (per-launch mean incl. boundaries)
// and 20 single launches bracketed by hipExtLaunchKernel events (device time).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__global__ void copy_kernel(const float4 *__restrict__ in, float4 *__restrict__ out, size_t nr, size_t nw) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    float4 acc = make_float4(0, 0, 0, 0);
    for (size_t k = i; k < nr; k += stride) {
        float4 v = in[k];
        acc.x += v.x;
        acc.y += v.y;
    }
    for (size_t k = i; k < nw; k += stride) out[k] = acc;
}

__global__ void store_f64(double *__restrict__ out, size_t n, double v) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = i; k < n; k += stride) out[k] = v + (double)k;
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__global__ void store_msk(double *__restrict__ out, size_t n, uint32_t thresh) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    for (size_t k = i; k < n; k += stride)
        if (hash((uint32_t)k) < thresh) out[k] = (double)k;
}

__global__ void load_msk(const double *__restrict__ in, double *__restrict__ out, size_t n, uint32_t thresh) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    double acc = 0;
    for (size_t k = i; k < n; k += stride)
        if (hash((uint32_t)k) < thresh) acc += in[k];
    if (acc == 12345.0) out[i] = acc;
}

template <class F>
void timeit(const char *name, double bytes, F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; ++i) launch(nullptr, nullptr);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a, 0));
    const int R = 200;
    for (int i = 0; i < R; ++i) launch(nullptr, nullptr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double per = ms / R * 1e3;
    double dev = 0;
    for (int i = 0; i < 20; ++i) {
        launch(a, b);
        CK(hipEventSynchronize(b));
        float m;
        CK(hipEventElapsedTime(&m, a, b));
        dev += m * 1e3 / 20;
    }
    printf("%-34s %10.1f MB  back-to-back %8.2f us (%7.1f GB/s)  device %8.2f us (%7.1f GB/s)\n", name, bytes / 1e6,
           per, bytes / per / 1e3, dev, bytes / dev / 1e3);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const size_t MB = 1 << 20;
    void *bufA, *bufB;
    CK(hipMalloc(&bufA, 512 * MB));
    CK(hipMalloc(&bufB, 512 * MB));
    CK(hipMemset(bufA, 0, 512 * MB));
    CK(hipMemset(bufB, 0, 512 * MB));
    const int block = 256;
    for (double rmb : {17.5, 35.0, 70.0}) {
        const double wmb = rmb * 14.5 / 17.5;
        const size_t nr = (size_t)(rmb * 1e6 / 16), nw = (size_t)(wmb * 1e6 / 16);
        for (int grid : {1024, 2048, 4096}) {
            char nm[64];
            snprintf(nm, sizeof nm, "copy r%.1f w%.1f g%d", rmb, wmb, grid);
            timeit(nm, (nr + nw) * 16.0, [&](hipEvent_t s, hipEvent_t e) {
                hipExtLaunchKernelGGL(copy_kernel, dim3(grid), dim3(block), 0, 0, s, e, 0, (const float4 *)bufA,
                                      (float4 *)bufB, nr, nw);
            });
        }
    }
    for (double mb : {63.0, 126.0, 189.0}) {
        const size_t n = (size_t)(mb * 1e6 / 8);
        char nm[64];
        snprintf(nm, sizeof nm, "store_f64 %.0fMB", mb);
        timeit(nm, n * 8.0, [&](hipEvent_t s, hipEvent_t e) {
            hipExtLaunchKernelGGL(store_f64, dim3(8192), dim3(block), 0, 0, s, e, 0, (double *)bufA, n, 1.0);
        });
    }
    for (double p : {0.12, 0.4, 0.7, 0.95, 1.0}) {
        const size_t n = (size_t)(126e6 / 8);
        const uint32_t th = p >= 1.0 ? 0xffffffffu : (uint32_t)(p * 4294967296.0);
        char nm[64];
        snprintf(nm, sizeof nm, "store_msk p=%.2f (126MB span)", p);
        timeit(nm, n * 8.0, [&](hipEvent_t s, hipEvent_t e) {
            hipExtLaunchKernelGGL(store_msk, dim3(8192), dim3(block), 0, 0, s, e, 0, (double *)bufA, n, th);
        });
        snprintf(nm, sizeof nm, "load_msk  p=%.2f (126MB span)", p);
        timeit(nm, n * 8.0, [&](hipEvent_t s, hipEvent_t e) {
            hipExtLaunchKernelGGL(load_msk, dim3(8192), dim3(block), 0, 0, s, e, 0, (const double *)bufA,
                                  (double *)bufB, n, th);
        });
    }
    return 0;
}
