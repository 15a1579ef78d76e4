// sng_kernels.hip -- HIP kernels of the batched SmartNanogridEnv hot path (gfx950).
//
// One thread = one environment; one 64-thread workgroup = one wavefront = 64 envs.
// Per-env state is SoA with the env index fastest (sng_layout.h), so every per-charger
// load/store of a wavefront is one contiguous 256 B (u32) or 512 B (f64) run.
// The policy-facing row-major actions [E][A] and observations [E][O] are staged
// through LDS so the HBM side of both is a contiguous, 16-byte-per-lane stream.
//
// Arithmetic follows the reference operation for operation (no FMA contraction:
// built with -ffp-contract=off); see the per-line citations.  Sums over chargers use
// the same order as the reference: numpy's pairwise sum for the charging powers
// (charging_station.py:293-294) and Python's left-to-right sum() for penalties
// (penaliser.py:55).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sng_layout.h"
#include "sng.h"

namespace sng {

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------
// numpy pairwise_sum (loops_utils.h.src) for n <= 128, fed one element at a time in
// array order.  Elements are buffered per block of 8; a block that completes is folded
// into the 8 running accumulators, the last partial block is the sequential tail.
// ---------------------------------------------------------------------------------
struct PairwiseSum {
    double r[8];
    double b[8];
    int n;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int q = 0; q < 8; ++q) { r[q] = 0.0; b[q] = 0.0; }
        n = 0;
    }
    __device__ __forceinline__ void push(double x) {
        const int j = n & 7;
#pragma unroll
        for (int q = 0; q < 8; ++q) b[q] = (q == j) ? x : b[q];
        ++n;
        if ((n & 7) == 0) {
            const bool first = (n == 8);
#pragma unroll
            for (int q = 0; q < 8; ++q) r[q] = first ? b[q] : r[q] + b[q];
        }
    }
    __device__ __forceinline__ double result() const {
        const int tail = n & 7;
        double res = (n < 8) ? 0.0 : ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (q < tail) res += b[q];
        return res;
    }
};

__device__ __forceinline__ size_t lds_obs_offset(int act_dim) {
    // obs staging area starts after the actions, rounded to 16 bytes
    return ((size_t)kWave * act_dim + 3) & ~(size_t)3;
}

// Copy `count` floats global -> LDS with 16 B per lane when the run is aligned.  Each lane
// issues up to K loads before the first LDS write, so the whole copy is one HBM round trip
// when count <= K * 256 floats.
template <int K>
__device__ __forceinline__ void copy_in(float *__restrict__ dst, const float *__restrict__ src, int count,
                                        bool vec, int lane) {
    if (vec && (count & 3) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        const int n4 = count >> 2;
        for (int base = 0; base < n4; base += K * kWave) {
            float4 v[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {   // clamped, unconditional: no per-element branch + wait
                const int i = base + k * kWave + lane;
                v[k] = s4[i < n4 ? i : n4 - 1];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {   // out-of-range lanes rewrite the last element (same value)
                const int i = base + k * kWave + lane;
                d4[i < n4 ? i : n4 - 1] = v[k];
            }
        }
    } else {
        for (int base = 0; base < count; base += 4 * K * kWave) {
            float v[4 * K];
#pragma unroll
            for (int k = 0; k < 4 * K; ++k) {
                const int i = base + k * kWave + lane;
                v[k] = src[i < count ? i : count - 1];
            }
#pragma unroll
            for (int k = 0; k < 4 * K; ++k) {
                const int i = base + k * kWave + lane;
                dst[i < count ? i : count - 1] = v[k];
            }
        }
    }
}

__device__ __forceinline__ void copy_out(float *__restrict__ dst, const float *__restrict__ src, int count,
                                         bool vec, int lane) {
    if (vec && (count & 3) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        for (int i = lane; i < (count >> 2); i += kWave) d4[i] = s4[i];
    } else {
        for (int i = lane; i < count; i += kWave) dst[i] = src[i];
    }
}

// Observation header (smart_nanogrid_environment.py:199-240, central_management_system.py:53-60):
// [solar(t), price(t), solar(t+1..t+3), price(t+1..t+3)] with PV, [price(t), price(t+1..t+3)] without.
__device__ __forceinline__ int write_obs_header(float *o, const Params &p, const Tables *tb, int t, double ratio) {
    int k = 0;
    if (p.pv) o[k++] = (float)(tb->irr_norm[t] * ratio);
    o[k++] = (float)tb->price_norm[t];
    if (p.pv) {
#pragma unroll
        for (int j = 1; j <= 3; ++j) o[k++] = (float)(tb->irr_norm[t + j] * ratio);
    }
#pragma unroll
    for (int j = 1; j <= 3; ++j) o[k++] = (float)tb->price_norm[t + j];
    return k;
}

// ---------------------------------------------------------------------------------
// The fused step: SmartNanogridEnv.step(actions) for 64 envs per workgroup.
// NC   = compile-time charger count (0: runtime p.n);
// DIAG = also write the per-step diagnostics (SngInfo arrays).
// All per-charger loads of a batch of CH chargers are issued before any of them is used
// (and the first batch before the action staging wait), so a wavefront keeps
// 3*CH + 2 independent HBM requests in flight instead of one round trip per charger.
// ---------------------------------------------------------------------------------
template <int NC, bool DIAG>
__global__ __launch_bounds__(kWave) void step_kernel(Params p, DeviceState s, InfoPtrs info,
                                                     const float *__restrict__ act, float *__restrict__ obs,
                                                     double *__restrict__ reward, uint8_t *__restrict__ done,
                                                     int64_t E, int t, int vec_io) {
    constexpr int CH = (NC > 0 && NC <= 16) ? NC : 8;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = NC ? NC : p.n;
    const int A = p.act_dim, O = p.obs_dim;
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int nblk = (int)((E - e0) < kWave ? (E - e0) : kWave);
    const int64_t e = e0 + lane;
    const bool live = lane < nblk;
    float *s_act = lds;
    float *s_obs = lds + lds_obs_offset(A);
    const uint32_t *__restrict__ word = s.word;
    const double *__restrict__ auxv = s.aux;
    double *__restrict__ socv = s.soc;
    const size_t tbase = (size_t)t * n;

    uint32_t w[CH];
    double aux[CH], run[CH];
    auto load_batch = [&](int c0) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int c = c0 + j;
            if (c < n) {
                const size_t idx = (tbase + c) * (size_t)E + e;
                w[j] = word[idx];
                aux[j] = auxv[idx];
                run[j] = socv[(size_t)c * E + e];
            }
        }
    };

    double ratio = 0.0, bess = 0.0;
    if (live) {
        ratio = s.ratio[e];
        if (p.bess) bess = s.bess[e];
        load_batch(0);
    }
    copy_in<(NC > 0 && NC < 16) ? 4 : 8>(s_act, act + e0 * A, nblk * A, vec_io != 0, lane);
    __syncthreads();

    if (live) {
        const Tables *tb = s.tables;
        const float *a_row = s_act + lane * A;
        float *o_row = s_obs + lane * O;
        const int k_soc = (p.pv ? 8 : 4);
        const int k_dep = k_soc + n;

        PairwiseSum pos, neg;
        pos.init();
        neg.init();
        double pen_v = 0.0, nonexist = 0.0;
        uint32_t fl = 0;
        for (int c0 = 0; c0 < n; c0 += CH) {
            if (c0 > 0) load_batch(c0);
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int c = c0 + j;
                if (c >= n) break;
                const uint32_t wj = w[j];
                double r = run[j];
                const float a = a_row[c];

                // penalise_charging_vehicles_outside_bounds (penaliser.py:39-57, 71-87): the vehicle's
                // SoC and requested SoC at python index t-1; Python sum() order over the list.
                if (t > 0 && (wj & W_PEN)) {
                    const double req = p.req_stream ? s.req[(tbase + c) * (size_t)E + e] : 1.0;
                    const double margin = 0.05 * req;
                    if (r < req - margin) {
                        const double d = (req - r) * 10;
                        pen_v += d * d;
                    }
                }

                // Charger.charge_or_discharge_vehicle (charger.py:37-56, 58-94, 108-144)
                double pw = 0.0;
                if (wj & W_OCC) {
                    const double prev = (wj & W_STATIC) ? aux[j] : r;
                    const double cap = (double)((wj >> W_CAP_SHIFT) & 0xffu);
                    double nsoc = prev;
                    if (a == 0.0f) {
                        nsoc = prev;
                    } else if (!p.bounded) {
                        fl |= SNG_FLAG_CHARGING_MODE;
                    } else {
                        double pc, change;
                        if (p.legacy) {               // NumPy < 2: float32 scalar * int -> float64
                            pc = ((double)a * p.ev_power) * p.ev_eff;
                            change = (pc * p.dt) / cap;
                        } else {                      // NumPy 2 (NEP 50): float32 product
                            const float pf = __fmul_rn(__fmul_rn(a, p.ev_power_f), p.ev_eff_f);
                            const float pdt = __fmul_rn(pf, p.dt_f);
                            pc = (double)pf;
                            change = (double)pdt / cap;
                        }
                        const double calc = prev + change;
                        if (a > 0.0f) {
                            nsoc = (1.0 < calc) ? 1.0 : calc;                     // min(calc, 1.0)
                            pw = pc;                                              // full power billed
                        } else {
                            pw = (calc >= 0.0) ? -((prev * cap) / p.dt) : pc;     // inverted flag, :122-132
                            nsoc = (calc > 0.0) ? calc : 0.0;                     // max(0.0, calc)
                        }
                    }
                    r = nsoc;
                } else {
                    if (a != 0.0f) nonexist += 100.0;                             // reset_info_values, :146-156
                    r = aux[j];                                                   // SOC[c, t] of an empty charger
                }
                socv[(size_t)c * E + e] = r;
                if (pw > 0.0) pos.push(pw);
                if (pw < 0.0) neg.push(pw);

                o_row[k_soc + c] = (float)r;
                o_row[k_dep + c] = (float)((double)((wj >> W_DEP_SHIFT) & 0xffu) / 24);
            }
        }
        if (t == 0) pen_v = s.pen0[e];

        const double p_dis = neg.result();                                   // charging_station.py:293
        const double p_ch = pos.result();                                    // :294
        const double solar = p.pv ? tb->pv_power[t] * ratio : 0.0;           // central_management_system.py:99-103
        const double demand = p_ch + p_dis;                                  // :105
        if (demand < 0.0) fl |= p.v2x ? SNG_FLAG_V2X_BREAKPOINT : SNG_FLAG_NEGATIVE_DEMAND;
        double rem = demand - solar;                                         // :167

        // BatteryEnergyStorageSystem.charge_or_discharge (battery_energy_storage_system.py:186-262)
        double pen_b = 0.0, bpow = 0.0, bcalc = 0.0;
        if (p.bess) {
            if (t == 0) s.bess0[e] = bess;                                   // :93-94
            const double ba = (double)a_row[n];
            if (ba == 0.0) {
                bpow = 0.0;
                bcalc = 0.0;
            } else if (!p.bounded) {
                fl |= SNG_FLAG_CHARGING_MODE;
            } else if (ba > 0.0) {
                const double avail = -rem;
                const double cp = (ba * p.bess_pmax_ch) * p.bess_eff_ch;
                const double calc = bess + (cp * p.dt) / p.bess_cap;
                bcalc = cp;
                bess = (1.0 < calc) ? 1.0 : calc;
                bpow = cp;
                rem = -(avail - cp);
            } else {
                double dp = (ba * p.bess_pmax_dis) * p.bess_eff_dis;
                const double calc = bess + (dp * p.dt) / p.bess_cap;
                bcalc = dp;
                if (calc < 0.0) dp = -((bess * p.bess_cap) / p.dt);
                bess = (calc > 0.0) ? calc : 0.0;
                bpow = dp;
                rem = rem + dp;
            }
            // penalise_battery_state_below_depth_of_discharge (penaliser.py:104-111)
            if (bess < p.bess_dod) {
                const double d = (p.bess_dod - bess) * 10;
                pen_b = d * d;
            } else if (!(bess <= 1.0)) {
                fl |= SNG_FLAG_BESS_SOC_ABOVE_1;
            }
            s.bess[e] = bess;
        }

        // Accountant (accountant.py:213-227) and Penaliser totals (penaliser.py:177-187)
        const double grid = rem;
        const double energy = grid * p.dt;
        const double price = tb->price[t];
        const double cost = (energy < 0.0) ? (energy * p.sell_coef) * price : energy * price;
        const double tot_pen = p.bat_pen_w * pen_b + pen_v;
        const double total = p.grid_w * fabs(cost) + tot_pen;
        reward[e] = -total;
        done[e] = (t + 1 == p.T) ? 1 : 0;

        write_obs_header(o_row, p, tb, t, ratio);
        if (p.bess) o_row[k_dep + n] = (float)bess;

        if (fl) s.flags[e] |= fl;
        if (info.flags) info.flags[e] = fl;
        if (info.episode_return) info.episode_return[e] += -total;
        if (DIAG) {
            if (info.grid_power) info.grid_power[e] = grid;
            if (info.p_charge) info.p_charge[e] = p_ch;
            if (info.p_discharge) info.p_discharge[e] = p_dis;
            if (info.bess_soc) info.bess_soc[e] = p.bess ? bess : 0.0;
            if (info.pen_vehicle) info.pen_vehicle[e] = pen_v;
            if (info.pen_battery) info.pen_battery[e] = pen_b;
            if (info.grid_cost) info.grid_cost[e] = cost;
            if (info.total_cost) info.total_cost[e] = total;
            if (info.solar) info.solar[e] = solar;
            if (info.bess_power) info.bess_power[e] = bpow;
            if (info.bess_calc_power) info.bess_calc_power[e] = bcalc;
            if (info.nonexistent) info.nonexistent[e] = nonexist;
            if (info.bess_initial) info.bess_initial[e] = p.bess ? s.bess0[e] : 0.0;
        }
    }
    __syncthreads();
    copy_out(obs + e0 * O, s_obs, nblk * O, vec_io != 0, lane);
}

// ---------------------------------------------------------------------------------
// Observation at t = 0 after a reset (SmartNanogridEnv.reset -> __get_observations,
// smart_nanogrid_environment.py:358-360): SOC[c, 0] as generated, departure times at 0.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kWave) void observe0_kernel(Params p, DeviceState s, float *__restrict__ obs,
                                                         double *__restrict__ ep_return, int64_t E, int vec_io) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = p.n, O = p.obs_dim;
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * kWave;
    const int nblk = (int)((E - e0) < kWave ? (E - e0) : kWave);
    const int64_t e = e0 + lane;
    float *o_row = lds + lane * O;
    if (lane < nblk) {
        const double ratio = s.ratio[e];
        int k = write_obs_header(o_row, p, s.tables, 0, ratio);
        for (int c = 0; c < n; ++c) {
            const size_t idx = (size_t)c * E + e;   // t = 0 slice
            const double aux = s.aux[idx];
            s.soc[idx] = aux;
            o_row[k + c] = (float)aux;
            o_row[k + n + c] = (float)((double)((s.word[idx] >> W_DEP_SHIFT) & 0xffu) / 24);
        }
        if (p.bess) o_row[k + 2 * n] = (float)s.bess[e];
        if (ep_return) ep_return[e] = 0.0;
    }
    if (blockIdx.x == 0 && lane == 0) *s.episode += 1;   // next Philox day
    __syncthreads();
    copy_out(obs + e0 * O, lds, nblk * O, vec_io != 0, lane);
}

// ---------------------------------------------------------------------------------
// Device RNG day generator (same distributions as charging_station.py:200-279, Philox
// draws).  Thread = (env, charger); writes the dense word/aux(/req) timeline.
// ---------------------------------------------------------------------------------
struct Philox {
    uint32_t k0, k1;
    __device__ __forceinline__ uint4 operator()(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) const {
        uint32_t key0 = k0, key1 = k1;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
            const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
            c0 = hi1 ^ c1 ^ key0;
            c1 = lo1;
            c2 = hi0 ^ c3 ^ key1;
            c3 = lo0;
            key0 += 0x9E3779B9u;
            key1 += 0xBB67AE85u;
        }
        return make_uint4(c0, c1, c2, c3);
    }
};

__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) / 9007199254740992.0;
}

__device__ __forceinline__ int below(uint32_t x, int n) {   // floor(x * n / 2^32)
    return (int)(((uint64_t)x * (uint64_t)n) >> 32);
}

__global__ __launch_bounds__(kWave) void generate_kernel(Params p, DeviceState s, uint64_t seed, int64_t E,
                                                         int i4, int i10, int i1) {
    const int64_t e = (int64_t)blockIdx.x * kWave + threadIdx.x;
    const int c = blockIdx.y;
    if (e >= E) return;
    const uint64_t day = *s.episode;
    const Philox rng{(uint32_t)seed, (uint32_t)(seed >> 32)};
    const uint32_t ce = (uint32_t)(e + p.env_offset), cday = (uint32_t)day;   // global env id
    uint32_t draw = 0;
    const int T = p.T, n = p.n;

    bool present = false, prev_occ = false;
    int dep = 0, prev_rem = 0;
    uint32_t cap = 0;
    double req = 0.0;
    for (int t = 0; t < T; ++t) {
        bool arrived = false;
        double soc_arr = 0.0;
        if (!present) {
            const uint4 x = rng(draw++, (uint32_t)c, ce, cday);
            if ((u53(x.x, x.y) - 0.1) > 0.5) {                      // round(rand() - 0.1) == 1
                arrived = true;
                present = true;
                soc_arr = 0.1 + (0.9 - 0.1) * u53(x.z, x.w);       // uniform(0.1, 0.9)
                const uint4 y = rng(draw++, (uint32_t)c, ce, cday);
                cap = p.diff_caps ? (uint32_t)(15 + below(y.x, 105)) : 40u;   // randint(15, 120)
                if (p.req_enabled) {
                    const double lo = soc_arr <= 0.9 ? soc_arr + 0.1 : 1.0;
                    req = lo + (1.0 - lo) * u53(y.z, y.w);
                } else {
                    req = 1.0;
                }
                const int hi_c = t + i10, hi_d = T + i1;
                const int high = hi_c < hi_d ? hi_c : hi_d;
                const int low = t + i4;
                dep = (low >= high) ? low : low + below(y.y, high - low);
            }
        }
        const bool occ = present && t < dep;
        if (!occ) present = false;
        // penalty-check list built by observe(t-1) (charging_station.py:42-63)
        bool pen = false;
        if (t > 0 && prev_occ) {
            switch (p.penalty_mode) {
                case SNG_PENALTY_ON_DEPARTURE: pen = (prev_rem == 1); break;
                case SNG_PENALTY_SPARSE: pen = (prev_rem >= 1 && prev_rem <= 3); break;
                case SNG_PENALTY_DENSE: pen = true; break;
                default: pen = false;
            }
        }
        const int rem = occ ? dep - t : 0;
        const size_t idx = ((size_t)t * n + c) * (size_t)E + e;
        s.word[idx] = pack_word(occ, arrived, pen, occ ? cap : 0u, (uint32_t)rem);
        if (arrived || !occ) s.aux[idx] = arrived ? soc_arr : 0.0;
        if (p.req_stream && pen) s.req[idx] = req;
        prev_occ = occ;
        prev_rem = rem;
    }
    if (c == 0) {
        const uint4 z = rng(0xFFFFFFFFu, 0xFFFFFFFFu, ce, cday);
        s.ratio[e] = (double)below(z.x, 181) / 100;                 // random.randint(0, 180) / 100
        s.pen0[e] = 0.0;
    }
}

// ---------------------------------------------------------------------------------
// launch wrappers (called from sng_api.cpp)
// ---------------------------------------------------------------------------------
size_t step_lds_bytes(const Params &p) {
    return (((size_t)kWave * p.act_dim + 3) & ~(size_t)3) * 4 + (size_t)kWave * p.obs_dim * 4;
}

// Optional start/stop events (ev != nullptr): hipExtLaunchKernel stamps them with the
// dispatch's own begin/end timestamps, i.e. the kernel's device time.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};

template <int NC, bool DIAG>
static void launch_step_t(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                          double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                          const LaunchEvents *ev) {
    const dim3 grid((unsigned)((E + kWave - 1) / kWave)), block(kWave);
    if (ev)
        hipExtLaunchKernelGGL((step_kernel<NC, DIAG>), grid, block, (uint32_t)step_lds_bytes(p), stream, ev->start,
                              ev->stop, 0u, p, s, info, act, obs, reward, done, E, t, vec_io);
    else
        hipLaunchKernelGGL((step_kernel<NC, DIAG>), grid, block, step_lds_bytes(p), stream, p, s, info, act, obs,
                           reward, done, E, t, vec_io);
}

template <bool DIAG>
static void launch_step_n(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                          double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                          const LaunchEvents *ev) {
    switch (p.n) {
        case 1: launch_step_t<1, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 2: launch_step_t<2, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 4: launch_step_t<4, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 8: launch_step_t<8, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 10: launch_step_t<10, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 16: launch_step_t<16, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 50: launch_step_t<50, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        default: launch_step_t<0, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
    }
}

hipError_t launch_step(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                       double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                       hipEvent_t ev_start, hipEvent_t ev_stop) {
    LaunchEvents evs{ev_start, ev_stop};
    const LaunchEvents *ev = (ev_start && ev_stop) ? &evs : nullptr;
    const bool diag = info.grid_power || info.p_charge || info.p_discharge || info.bess_soc || info.pen_vehicle ||
                      info.pen_battery || info.grid_cost || info.total_cost || info.solar || info.bess_power ||
                      info.bess_calc_power || info.nonexistent || info.bess_initial;
    if (diag)
        launch_step_n<true>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev);
    else
        launch_step_n<false>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev);
    return hipGetLastError();
}

hipError_t launch_observe0(const Params &p, const DeviceState &s, float *obs, double *ep_return, int64_t E,
                           int vec_io, hipStream_t stream) {
    const dim3 grid((unsigned)((E + kWave - 1) / kWave)), block(kWave);
    const size_t lds = (size_t)kWave * p.obs_dim * 4;
    hipLaunchKernelGGL(observe0_kernel, grid, block, lds, stream, p, s, obs, ep_return, E, vec_io);
    return hipGetLastError();
}

hipError_t launch_generate(const Params &p, const DeviceState &s, uint64_t seed, int64_t E, int i4, int i10, int i1,
                           hipStream_t stream) {
    const dim3 grid((unsigned)((E + kWave - 1) / kWave), (unsigned)p.n), block(kWave);
    hipLaunchKernelGGL(generate_kernel, grid, block, 0, stream, p, s, seed, E, i4, i10, i1);
    return hipGetLastError();
}

}  // namespace sng
