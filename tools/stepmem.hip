// stepmem.hip -- the step kernel's memory traffic with trivial arithmetic, per state layout.
// Not part of the product.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/stepmem tools/stepmem.hip
//
// Per env-step (N chargers): actions (N+1) f32 in, observation 2N+9 f32 out (through LDS, 16 B
// stores), reward f64 + done u8 out, BESS f64 r/w, PV ratio f64 in, day return f64 r/w, and per
// charger an 8 B scenario record in plus the f64 SoC r/w -- 36 N + 89 B, as the packed device day.
//
// Layouts of the per-charger planes (record timeline [T][...], SoC [...]):
//   soa   : [N][E]          charger rows E apart (the library's layout)
//   tile  : [E/64][N][64]   a wavefront's 64 envs x N chargers contiguous (5 KB per plane at N = 10)
// Each case: 24-launch "days" back to back (timeline records of step t), mean per launch.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int NC = 10;
constexpr int A = NC + 1, O = 2 * NC + 9;
typedef float v4f __attribute__((ext_vector_type(4)));

template <bool TILE, int BLOCK>
__global__ __launch_bounds__(BLOCK) void step_mem(const float *__restrict__ act, float *__restrict__ obs,
                                                 const uint64_t *__restrict__ rec, double *__restrict__ soc,
                                                 double *__restrict__ bess, const double *__restrict__ ratio,
                                                 double *__restrict__ ret, double *__restrict__ reward,
                                                 uint8_t *__restrict__ done, int64_t E, int t) {
    __shared__ __attribute__((aligned(16))) float s_act[BLOCK * A];
    __shared__ __attribute__((aligned(16))) float s_obs[BLOCK * O];
    const int tid = threadIdx.x, lane = tid & 63;
    const int64_t eb = (int64_t)blockIdx.x * BLOCK;
    const int64_t e = eb + tid;
    const int64_t w0 = e - lane;   // wavefront's first env
    const uint64_t *rec_t = rec + (size_t)t * NC * E;
    // per-env loads
    const double r = ratio[e], b = bess[e], rp = ret[e];
    // actions tile (16 B per lane)
    const v4f *a4 = reinterpret_cast<const v4f *>(act + eb * A);
    v4f av[(BLOCK * A / 4 + BLOCK - 1) / BLOCK];
#pragma unroll
    for (int k = 0; k < (BLOCK * A / 4 + BLOCK - 1) / BLOCK; ++k) {
        const int i = k * BLOCK + tid;
        av[k] = a4[i < BLOCK * A / 4 ? i : BLOCK * A / 4 - 1];
    }
    uint64_t rc[NC];
    double sc[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const size_t ix = TILE ? (size_t)w0 * NC + (size_t)c * 64 + lane : (size_t)c * E + e;
        rc[c] = rec_t[ix];
        sc[c] = soc[ix];
    }
#pragma unroll
    for (int k = 0; k < (BLOCK * A / 4 + BLOCK - 1) / BLOCK; ++k) {
        const int i = k * BLOCK + tid;
        reinterpret_cast<v4f *>(s_act)[i < BLOCK * A / 4 ? i : BLOCK * A / 4 - 1] = av[k];
    }
    __syncthreads();
    double pw = 0.0;
    float *orow = s_obs + tid * O;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const size_t ix = TILE ? (size_t)w0 * NC + (size_t)c * 64 + lane : (size_t)c * E + e;
        const float a = s_act[tid * A + c];
        const double x = sc[c] + (double)__uint_as_float((uint32_t)(rc[c] >> 32)) * (double)a;
        __builtin_nontemporal_store(x, &soc[ix]);
        pw += x;
        orow[8 + c] = (float)x;
        orow[8 + NC + c] = (float)(uint32_t)rc[c];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) orow[j] = (float)(r * j);
    const double nb = b + s_act[tid * A + NC] * 0.01;
    orow[O - 1] = (float)nb;
    __builtin_nontemporal_store(nb, &bess[e]);
    __builtin_nontemporal_store(-pw, &reward[e]);
    __builtin_nontemporal_store(rp - pw, &ret[e]);
    done[e] = (uint8_t)(t == 23);
    __syncthreads();
    v4f *o4 = reinterpret_cast<v4f *>(obs + eb * O);
    const v4f *so4 = reinterpret_cast<const v4f *>(s_obs);
    for (int i = tid; i < BLOCK * O / 4; i += BLOCK) __builtin_nontemporal_store(so4[i], &o4[i]);
}

template <bool TILE, int BLOCK>
void run(const char *name, int64_t E) {
    float *act, *obs;
    uint64_t *rec;
    double *soc, *bess, *ratio, *ret, *reward;
    uint8_t *done;
    const int T = 24;
    CK(hipMalloc(&act, E * A * 4 * (size_t)T));
    CK(hipMalloc(&obs, E * O * 4));
    CK(hipMalloc(&rec, (size_t)T * NC * E * 8));
    CK(hipMalloc(&soc, NC * E * 8));
    CK(hipMalloc(&bess, E * 8));
    CK(hipMalloc(&ratio, E * 8));
    CK(hipMalloc(&ret, E * 8));
    CK(hipMalloc(&reward, E * 8));
    CK(hipMalloc(&done, E));
    CK(hipMemset(act, 0, E * A * 4 * (size_t)T));
    CK(hipMemset(rec, 0, (size_t)T * NC * E * 8));
    CK(hipMemset(soc, 0, NC * E * 8));
    CK(hipMemset(bess, 0, E * 8));
    CK(hipMemset(ratio, 0, E * 8));
    CK(hipMemset(ret, 0, E * 8));
    const dim3 grid((unsigned)(E / BLOCK)), block(BLOCK);
    auto day = [&](hipEvent_t *ev) {
        for (int t = 0; t < T; ++t) {
            hipExtLaunchKernelGGL((step_mem<TILE, BLOCK>), grid, block, 0, 0, ev ? ev[2 * t] : nullptr,
                                  ev ? ev[2 * t + 1] : nullptr, 0, act + (size_t)t * E * A, obs, rec, soc, bess,
                                  ratio, ret, reward, done, E, t);
        }
    };
    for (int i = 0; i < 5; ++i) day(nullptr);
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int D = 20;
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < D; ++i) day(nullptr);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<hipEvent_t> ev(2 * T);
    for (auto &x : ev) CK(hipEventCreate(&x));
    double dev = 0;
    const int DD = 3;
    for (int i = 0; i < DD; ++i) {
        day(ev.data());
        CK(hipDeviceSynchronize());
        for (int t = 0; t < T; ++t) {
            float m;
            CK(hipEventElapsedTime(&m, ev[2 * t], ev[2 * t + 1]));
            dev += m * 1e3;
        }
    }
    dev /= DD * T;
    const double per = ms * 1e3 / (D * T);
    const double bytes = (double)E * (36 * NC + 89);
    printf("%-22s E=%7lld  back-to-back %6.2f us/launch (%6.0f GB/s)  device %6.2f us (%6.0f GB/s)\n", name,
           (long long)E, per, bytes / per / 1e3, dev, bytes / dev / 1e3);
    for (auto &x : ev) CK(hipEventDestroy(x));
    CK(hipFree(act));
    CK(hipFree(obs));
    CK(hipFree(rec));
    CK(hipFree(soc));
    CK(hipFree(bess));
    CK(hipFree(ratio));
    CK(hipFree(ret));
    CK(hipFree(reward));
    CK(hipFree(done));
}

int main() {
    for (int rep = 0; rep < 2; ++rep) {
        for (int64_t E : {65536LL, 262144LL}) {
            run<false, 256>("soa  wg256", E);
            run<true, 256>("tile wg256", E);
            run<false, 64>("soa  wg64", E);
            run<true, 64>("tile wg64", E);
        }
    }
    return 0;
}
