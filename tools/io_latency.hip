// Host round-trip latency of one small step, the shape of SmartNanogridEnv.step (one env: 44 B of actions in,
// ~130 B of reward / observation / done out, one flag word), measured for the ways the host can drive it:
//   kernel        the kernel alone + hipStreamSynchronize (the floor of any host-driven step)
//   copies        pinned H2D copy, kernel, pinned D2H copy, synchronize (what SmartNanogridEnv.step does)
//   copies2       the same with a second D2H copy (a separate flag word)
//   zerocopy      the kernel reads the actions from and writes the outputs to pinned host memory
//                 (hipHostMalloc, mapped) directly: one command + synchronize
//   zerocopy_nc   the same with hipHostMallocNonCoherent memory
//   memcpy_sync   hipMemcpy H2D, kernel, hipMemcpy D2H (blocking copies)
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/io_latency tools/io_latency.hip
// Prints the median and 90th percentile per round trip in microseconds, 20,000 round trips per mode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int kAct = 11, kObs = 29;

// a stand-in step: reads the actions, writes reward, observation and done (one wavefront)
__global__ void tiny_step(const float *act, double *rew, float *obs, unsigned char *done, int t) {
    const int l = threadIdx.x;
    float a = l < kAct ? act[l] : 0.f;
    for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
    if (l < kObs) obs[l] = a * (float)(l + 1);
    if (l == 0) {
        rew[0] = -(double)a;
        done[0] = (unsigned char)(t == 23);
    }
}

using clk = std::chrono::steady_clock;

static void report(const char *name, std::vector<double> &us) {
    std::sort(us.begin(), us.end());
    std::printf("%-12s median %7.2f us  p90 %7.2f us  min %7.2f us\n", name, us[us.size() / 2], us[us.size() * 9 / 10],
                us[0]);
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 20000;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    float *act_d, *obs_d;
    double *rew_d;
    unsigned char *done_d;
    unsigned *flag_d;
    CK(hipMalloc(&act_d, 256));
    CK(hipMalloc(&obs_d, 256));
    CK(hipMalloc(&rew_d, 256));
    CK(hipMalloc(&done_d, 256));
    CK(hipMalloc(&flag_d, 256));
    CK(hipMemset(flag_d, 0, 256));
    // pinned staging: [actions 64 B | reward 8 | obs 116 | done 1] as one block for one D2H copy
    char *pin;
    CK(hipHostMalloc(&pin, 4096, hipHostMallocDefault));
    char *blk_d;
    CK(hipMalloc(&blk_d, 4096));
    char *map_c, *map_nc;
    CK(hipHostMalloc(&map_c, 4096, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(&map_nc, 4096, hipHostMallocMapped | hipHostMallocNonCoherent));
    float act[kAct];
    for (int i = 0; i < kAct; ++i) act[i] = 0.1f * i;
    std::vector<double> us(n);
    auto run = [&](const char *name, auto &&body) {
        for (int i = 0; i < 200; ++i) body(i);
        for (int i = 0; i < n; ++i) {
            auto t0 = clk::now();
            body(i);
            us[i] = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        }
        report(name, us);
    };
    run("kernel", [&](int i) {
        tiny_step<<<1, 64, 0, st>>>(act_d, rew_d, obs_d, done_d, i % 24);
        CK(hipStreamSynchronize(st));
    });
    run("copies", [&](int i) {
        std::memcpy(pin, act, sizeof act);
        CK(hipMemcpyAsync(blk_d, pin, sizeof act, hipMemcpyHostToDevice, st));
        tiny_step<<<1, 64, 0, st>>>((const float *)blk_d, (double *)(blk_d + 64), (float *)(blk_d + 72),
                                    (unsigned char *)(blk_d + 188), i % 24);
        CK(hipMemcpyAsync(pin + 64, blk_d + 64, 128, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    run("copies2", [&](int i) {
        std::memcpy(pin, act, sizeof act);
        CK(hipMemcpyAsync(blk_d, pin, sizeof act, hipMemcpyHostToDevice, st));
        tiny_step<<<1, 64, 0, st>>>((const float *)blk_d, (double *)(blk_d + 64), (float *)(blk_d + 72),
                                    (unsigned char *)(blk_d + 188), i % 24);
        CK(hipMemcpyAsync(pin + 64, blk_d + 64, 128, hipMemcpyDeviceToHost, st));
        CK(hipMemcpyAsync(pin + 256, flag_d, 4, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    for (int nc = 0; nc < 2; ++nc) {
        char *m = nc ? map_nc : map_c;
        char *md;
        CK(hipHostGetDevicePointer((void **)&md, m, 0));
        run(nc ? "zerocopy_nc" : "zerocopy", [&](int i) {
            std::memcpy(m, act, sizeof act);
            tiny_step<<<1, 64, 0, st>>>((const float *)md, (double *)(md + 64), (float *)(md + 72),
                                        (unsigned char *)(md + 188), i % 24);
            CK(hipStreamSynchronize(st));
            if (((double *)(m + 64))[0] == 1234.5) std::printf("?");
        });
        // correctness of the zero-copy outputs
        std::memset(m + 64, 0, 128);
        tiny_step<<<1, 64, 0, st>>>((const float *)md, (double *)(md + 64), (float *)(md + 72), (unsigned char *)(md + 188), 23);
        CK(hipStreamSynchronize(st));
        float s = 0;
        for (int k = 0; k < kAct; ++k) s += act[k];
        std::printf("  %s check: reward %.6f (expect %.6f) obs[1] %.6f done %d\n", nc ? "zerocopy_nc" : "zerocopy",
                    ((double *)(m + 64))[0], -(double)s, ((float *)(m + 72))[1], (int)m[188]);
    }
    run("memcpy_sync", [&](int i) {
        CK(hipMemcpy(blk_d, act, sizeof act, hipMemcpyHostToDevice));
        tiny_step<<<1, 64, 0, st>>>((const float *)blk_d, (double *)(blk_d + 64), (float *)(blk_d + 72),
                                    (unsigned char *)(blk_d + 188), i % 24);
        CK(hipMemcpyAsync(pin + 64, blk_d + 64, 128, hipMemcpyDeviceToHost, st));
        CK(hipStreamSynchronize(st));
    });
    CK(hipStreamDestroy(st));
    return 0;
}
