// sng_kernels.hip -- HIP kernels of the batched SmartNanogridEnv hot path (gfx950).
//
// Step kernel mapping: 256-thread workgroups (4 wavefronts); L lanes per environment
// (L = 1, 2 or 4), 256/L environments per workgroup.  Lane `part` of an env owns a
// contiguous range of chargers; the env's first lane (the leader) finishes the env (sums,
// BESS, cost, reward).  256-thread workgroups dispatch 4x fewer workgroups than one-wave
// groups (measured: the 1024 one-wave groups of a 65,536-env step took ~2 us just to start).
//
// Per-env state is SoA with the env index fastest (sng_layout.h), so every per-charger
// load/store of a wavefront is a contiguous run.  The policy-facing row-major actions
// [E][A] and observations [E][O] are staged through LDS so their HBM side is a contiguous,
// 16-byte-per-lane stream.
//
// Arithmetic follows the reference operation for operation (built with -ffp-contract=off;
// the two explicit fma-based divisions below are exact, see their comments).  Sums over
// chargers use the reference's order: numpy's pairwise sum for the charging powers
// (charging_station.py:293-294) and Python's left-to-right sum() for the vehicle penalties
// (penaliser.py:55).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "sng.h"
#include "sng_layout.h"

namespace sng {

constexpr int kWave = 64;

// Streaming (nontemporal) stores for the step's bulk outputs (SoC, observations): they leave
// less dirty L2 for the end-of-kernel release (measured 8.92 -> 8.17 us per step at 65,536 x 10).
#define SNG_ST(dst, v) __builtin_nontemporal_store((v), &(dst))
#include "sng_diag_hooks.h"   // empty hooks in libsng.so (tools/diag builds fill them)

// ---------------------------------------------------------------------------------
// numpy pairwise_sum (loops_utils.h.src) for n <= 128, fed one element at a time in
// array order (used for N > 16; smaller N use the LDS-compacted form below).
// ---------------------------------------------------------------------------------
struct PairwiseSum {
    double r[8];
    double b[8];
    int n;
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            r[q] = 0.0;
            b[q] = 0.0;
        }
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

// The same sum over a compacted array the lane has written to its own LDS row:
// n < 8 is the sequential sum `seq` the caller kept on the fly (adding the skipped +0.0
// terms is exact); otherwise 8 accumulators over full blocks, pairwise tree, sequential tail.
__device__ __forceinline__ double pairwise_row(const double *row, int n, double seq) {
    if (n < 8) return seq;
    double r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = row[j];
    const int full = n - (n & 7);
    for (int i = 8; i < full; i += 8) {
#pragma unroll
        for (int j = 0; j < 8; ++j) r[j] += row[i + j];
    }
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int i = full; i < n; ++i) res += row[i];
    return res;
}

// The same for a row of at most NC <= 16 entries: every slot is read in one batch of LDS reads
// (slots at or past n hold stale values and are selected away), so the sequential tail costs
// no LDS round trip per element.
template <int NC>
__device__ __forceinline__ double pairwise_row_c(const double *row, int n, double seq) {
    static_assert(NC >= 1 && NC <= 16, "one 8-block plus tail, or two full blocks at 16");
    if constexpr (NC < 8) {
        return seq;
    } else {
        if (n < 8) return seq;
        double r[NC];
#pragma unroll
        for (int j = 0; j < NC; ++j) r[j] = row[j];
        if (NC == 16 && n == 16) {
#pragma unroll
            for (int j = 0; j < 8; ++j) r[j] += r[(j + 8) % NC];
            return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        }
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int i = 8; i < NC; ++i) res = (i < n) ? res + r[i] : res;
        return res;
    }
}

__host__ __device__ constexpr int round4(int x) { return (x + 3) & ~3; }

// Raw buffer access: V# = an array (or a per-step timeline plane) in SGPRs, a wave-uniform
// byte offset (soffset, e.g. the charger row) and a per-lane 32-bit byte offset (the env).  The
// adds happen in the buffer unit instead of as 64-bit VALU adds per access.  Every array or plane
// addressed this way is < 4 GiB (checked at sng_create).  dword3 0x00020000: gfx9 raw buffer.
using Rsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ Rsrc rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, -1, 0x00020000);
}
constexpr int kNT = 2;   // buffer cache-policy bit: nontemporal (streaming) access
typedef unsigned v2u __attribute__((ext_vector_type(2)));
template <class T, int POL = 0>
__device__ __forceinline__ T bld(const T *base, uint32_t voff, uint32_t soff = 0) {
    static_assert(sizeof(T) == 4 || sizeof(T) == 8, "4 or 8 byte elements");
    if constexpr (sizeof(T) == 8)
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rsrc(base), voff, soff, POL));
    else
        return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rsrc(base), voff, soff, POL));
}
template <int POL = 0, class T>
__device__ __forceinline__ void bst(T *base, uint32_t voff, T v, uint32_t soff = 0) {
    static_assert(sizeof(T) == 1 || sizeof(T) == 4 || sizeof(T) == 8, "1, 4 or 8 byte elements");
    if constexpr (sizeof(T) == 8)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), rsrc(base), voff, soff, POL);
    else if constexpr (sizeof(T) == 4)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc(base), voff, soff, POL);
    else
        __builtin_amdgcn_raw_buffer_store_b8(__builtin_bit_cast(unsigned char, v), rsrc(base), voff, soff, POL);
}
// 2 B buffer accesses (the packed records of a device-RNG day, sng_layout.h), zero-extended.
__device__ __forceinline__ uint32_t bld16(const uint16_t *base, uint32_t voff, uint32_t soff = 0) {
    return (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rsrc(base), voff, soff, 0);
}
template <int POL = 0>
__device__ __forceinline__ void bst16(uint16_t *base, uint32_t voff, uint32_t v, uint32_t soff = 0) {
    __builtin_amdgcn_raw_buffer_store_b16((unsigned short)v, rsrc(base), voff, soff, POL);
}
// A device-RNG day's packed records (u16 [T+1][N][E] in the aux buffer) and a record's capacity field; a
// host-RNG or injected day's word carries it in bits 8-15 (sng_layout.h).
__device__ __forceinline__ const uint16_t *packed_records(const DeviceState &s) {
    return reinterpret_cast<const uint16_t *>(s.aux);
}
template <bool PK>
__device__ __forceinline__ uint32_t cap_field(uint32_t w) {
    return PK ? (w >> P_CAP_SHIFT) & P_CAP_MASK : (w >> W_CAP_SHIFT) & 0xffu;
}
// Byte offset of charger c of env el in a packed-record plane (charger quads, sng_layout.h rec_index): the
// per-lane part (v) and the wave-uniform quad row (s).
struct RecOff {
    uint32_t v, s;
};
__device__ __forceinline__ RecOff rec_off(int c, int n, int64_t E, uint32_t el) {
    const int c0 = c & ~3;
    const uint32_t w = (uint32_t)(n - c0 < 4 ? n - c0 : 4);
    return {(el * w + (uint32_t)(c & 3)) * 2u, (uint32_t)c0 * (uint32_t)E * 2u};
}
// The four records of one 8 B quad slot.
__device__ __forceinline__ void unpack_quad(uint64_t x, uint32_t *w) {
    w[0] = (uint32_t)x & 0xffffu;
    w[1] = (uint32_t)(x >> 16) & 0xffffu;
    w[2] = (uint32_t)(x >> 32) & 0xffffu;
    w[3] = (uint32_t)(x >> 48);
}
// Two f64 in one 16 B buffer access (a charger pair of the SoC state, sng_layout.h).
typedef unsigned v4u __attribute__((ext_vector_type(4)));
template <int POL = 0>
__device__ __forceinline__ void bld2(const double *base, uint32_t voff, uint32_t soff, double &a, double &b) {
    const v4u x = __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), voff, soff, POL);
    a = __builtin_bit_cast(double, (uint64_t)x.x | ((uint64_t)x.y << 32));
    b = __builtin_bit_cast(double, (uint64_t)x.z | ((uint64_t)x.w << 32));
}
// The wave-uniform offset goes into the V# base, not the soffset field: a MUBUF store of more than 8 B reads
// its data VGPRs a cycle late, and the compiler (ROCm 7.2 LLVM) inserts the wait state a VALU write of those
// VGPRs needs only when soffset is not a register.  gfx950 needs it either way: with an SGPR soffset, a
// v_cvt writing the pair's high dword right after the store corrupted ~0.1 % of the stored SoC slots at
// 65,536 envs (two waves per SIMD; tests/test_gpu_bench_kernel.py, tools/dbg/pairs_dbg.py).
template <int POL = 0>
__device__ __forceinline__ void bst2(double *base, uint32_t voff, double a, double b, uint32_t soff = 0) {
    const uint64_t ua = __builtin_bit_cast(uint64_t, a), ub = __builtin_bit_cast(uint64_t, b);
    const v4u x = {(unsigned)ua, (unsigned)(ua >> 32), (unsigned)ub, (unsigned)(ub >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(x, rsrc(reinterpret_cast<char *>(base) + soff), voff, 0, POL);
}
// Byte offset of charger c of the env whose 8 B slot offset is el8 (8 * env) in the SoC state (charger
// pairs, sng_layout.h soc_index), split into the per-lane part (v) and the wave-uniform part (s).
struct SocOff {
    uint32_t v, s;
};
__device__ __forceinline__ SocOff soc_off(int c, int n, int64_t E, uint32_t el8) {
    const int c0 = c & ~1;
    const bool two = c0 + 2 <= n;
    return {two ? 2u * el8 : el8, (uint32_t)c0 * (uint32_t)E * 8u + (two ? (uint32_t)(c & 1) * 8u : 0u)};
}

// Copy `count` floats global -> LDS with 16 B per lane when the run is aligned.  Each thread
// issues up to K loads before the first LDS write (clamped, unconditional loads: no per-element
// branch + wait), so the whole copy is one HBM round trip when count <= K * 4 * BLOCK floats.
template <int K, int BLOCK>
__device__ __forceinline__ void copy_in(float *__restrict__ dst, const float *__restrict__ src, int count,
                                        bool vec, int tid) {
    if (vec && (count & 3) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        const int n4 = count >> 2;
        for (int base = 0; base < n4; base += K * BLOCK) {
            float4 v[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = base + k * BLOCK + tid;
                v[k] = s4[i < n4 ? i : n4 - 1];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {   // out-of-range threads rewrite the last element (same value)
                const int i = base + k * BLOCK + tid;
                d4[i < n4 ? i : n4 - 1] = v[k];
            }
        }
    } else {
        for (int base = 0; base < count; base += 4 * K * BLOCK) {
            float v[4 * K];
#pragma unroll
            for (int k = 0; k < 4 * K; ++k) {
                const int i = base + k * BLOCK + tid;
                v[k] = src[i < count ? i : count - 1];
            }
#pragma unroll
            for (int k = 0; k < 4 * K; ++k) {
                const int i = base + k * BLOCK + tid;
                dst[i < count ? i : count - 1] = v[k];
            }
        }
    }
}

// The same copy split in two so other loads can be issued in between: issue() puts the
// block's tile in registers (one load per lane and k), commit() writes it to LDS.  When the
// tile does not fit one round (count > 4 * K * BLOCK floats) issue() does nothing and commit()
// falls back to copy_in.  Native vector types only (HIP's float4 wrapper keeps the array
// from being promoted to registers).
template <int K, int BLOCK>
struct TileStage {
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f v[K];
    const float *src;
    int count;
    bool vec, one_round;
    __device__ __forceinline__ void issue(const float *__restrict__ s, int cnt, bool vec_io, int tid) {
        src = s;
        count = cnt;
        vec = vec_io && (cnt & 3) == 0;
        one_round = vec ? (cnt >> 2) <= K * BLOCK : cnt <= K * BLOCK;
        if (!one_round) return;
        if (vec) {
            const v4f *s4 = reinterpret_cast<const v4f *>(s);
            const int n4 = cnt >> 2;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = k * BLOCK + tid;
                v[k] = s4[i < n4 ? i : n4 - 1];
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = k * BLOCK + tid;
                v[k].x = s[i < cnt ? i : cnt - 1];
            }
        }
    }
    __device__ __forceinline__ void commit(float *__restrict__ dst, int tid) {
        if (!one_round) {
            copy_in<K, BLOCK>(dst, src, count, vec, tid);
            return;
        }
        if (vec) {
            v4f *d4 = reinterpret_cast<v4f *>(dst);
            const int n4 = count >> 2;
#pragma unroll
            for (int k = 0; k < K; ++k) {   // out-of-range threads rewrite the last element (same value)
                const int i = k * BLOCK + tid;
                d4[i < n4 ? i : n4 - 1] = v[k];
            }
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const int i = k * BLOCK + tid;
                dst[i < count ? i : count - 1] = v[k].x;
            }
        }
    }
};

template <int BLOCK>
__device__ __forceinline__ void copy_out(float *__restrict__ dst, const float *__restrict__ src, int count,
                                         bool vec, int tid) {
    if (vec && (count & 3) == 0) {
        typedef float v4f __attribute__((ext_vector_type(4)));
        const v4f *s4 = reinterpret_cast<const v4f *>(src);
        v4f *d4 = reinterpret_cast<v4f *>(dst);
        for (int i = tid; i < (count >> 2); i += BLOCK) SNG_ST(d4[i], s4[i]);
    } else {
        for (int i = tid; i < count; i += BLOCK) dst[i] = src[i];
    }
}

// Observation header (smart_nanogrid_environment.py:190-231, central_management_system.py:53-60):
// [solar(t), price(t), solar(t+1..t+3), price(t+1..t+3)] with PV, [price(t), price(t+1..t+3)] without.
// irr / pn point at irr_norm[t] / price_norm[t] (the step kernel's LDS copy, or the tables);
// fpv / fpr are the env's profile factors for t..t+3 (1.0 without stochastic profiles).
__device__ __forceinline__ void write_obs_header(float *o, const Params &p, const double *irr, const double *pn,
                                                 double ratio, const double *fpv, const double *fpr) {
    int k = 0;
    if (p.pv) o[k++] = (float)((irr[0] * ratio) * fpv[0]);
    o[k++] = (float)(pn[0] * fpr[0]);
    if (p.pv) {
#pragma unroll
        for (int j = 1; j <= 3; ++j) o[k++] = (float)((irr[j] * ratio) * fpv[j]);
    }
#pragma unroll
    for (int j = 1; j <= 3; ++j) o[k++] = (float)(pn[j] * fpr[j]);
}

// ---------------------------------------------------------------------------------
// Counter-based 32-bit hash streams (device generator, stochastic profiles).  The oracle
// restates mix32 / stream_key / profile_factor bit for bit (oracle/sng_oracle.c).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {   // "triple32" integer hash (bijective)
    x ^= x >> 17;
    x *= 0xed5ad4bbu;
    x ^= x >> 11;
    x *= 0xac4c1b51u;
    x ^= x >> 15;
    x *= 0x31848babu;
    x ^= x >> 14;
    return x;
}

// Stream key of (seed, global env, charger | domain, day).
__device__ __forceinline__ uint32_t stream_key(uint64_t seed, uint64_t ge, uint32_t lane, uint64_t day) {
    const uint32_t k0 = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + (uint32_t)day * 0x9e3779b9u));
    const uint32_t k1 = mix32(k0 ^ (uint32_t)ge);
    return mix32(k1 ^ ((uint32_t)(ge >> 32) * 0x85ebca6bu + lane * 0xc2b2ae35u + 0x27d4eb2fu));
}

constexpr uint32_t kDomainPV = 0x50560000u;
constexpr uint32_t kDomainPrice = 0x50520000u;

// Build-defined stochastic profile factor 1 + sigma * z, z = h * 2^-31 - 1 in [-1, 1), of table
// entry k for the env with seed env_seed on day `day` (SngConfig.pv_noise / price_noise).
// The same from the day's key of the env and domain, stream_key(env_seed, 0, domain, day): what a reset keeps
// per env (DeviceState::prof_key) and the step kernels expand (round 4; round 3 stored every factor, 1.6 KB
// per env and day at config 5, and loaded 64 B per env-step).  sigma = 0 gives 1.0 exactly.
__device__ __forceinline__ double profile_factor_key(uint32_t key, int k, double sigma) {
    if (sigma == 0.0) return 1.0;
    const uint32_t h = mix32(key + (uint32_t)k * 0x9e3779b9u);
    const double z = (double)h * 0x1.0p-31 - 1.0;
    return 1.0 + sigma * z;
}
__device__ __forceinline__ double profile_factor(uint64_t env_seed, uint32_t domain, uint64_t day, int k,
                                                 double sigma) {
    return profile_factor_key(stream_key(env_seed, 0, domain, day), k, sigma);
}
// The day's profile keys of an env (PV, price) from DeviceState::prof_key ([E][2] u32, one 8 B load).
__device__ __forceinline__ void profile_factors(const Params &p, const DeviceState &s, uint32_t el8, int t,
                                                double *fpv, double *fpr) {
    const v2u kk = __builtin_bit_cast(v2u, bld(reinterpret_cast<const uint64_t *>(s.prof_key), el8));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        fpv[j] = profile_factor_key(kk.x, t + j, p.pv_noise);
        fpr[j] = profile_factor_key(kk.y, t + j, p.price_noise);
    }
}

// Per-step constants staged in LDS by the step kernel: irr_norm[t..t+3], price_norm[t..t+3],
// pv_power[t], price[t].
enum { CST_IRR = 0, CST_PN = 4, CST_PV = 8, CST_PRICE = 9, CST_COUNT = 10 };
__host__ __device__ inline double step_constant(const Tables *tb, int t, int i) {
    return i < CST_PN ? tb->irr_norm[t + i]
                      : i < CST_PV ? tb->price_norm[t + i - CST_PN] : i == CST_PV ? tb->pv_power[t] : tb->price[t];
}

// Remaining time to departure / 24 (smart_nanogrid_environment.py:207-208) as float32.
// The reference rounds d / 24 in float64 and then to float32; for integers d < 256 that equals the
// correctly rounded float32 quotient (d/24 is never a float32 rounding midpoint), which
// q = d*r; q + fma(-q, 24, d)*r reproduces for every d < 256 (checked exhaustively).
template <bool PK = false>   // PK: a packed record's steps-left field (bits 10-15; the record is zero-extended)
__device__ __forceinline__ float departure_obs(uint32_t w) {
    const float d = PK ? (float)(w >> P_DEP_SHIFT) : (float)((w >> W_DEP_SHIFT) & 0xffu);
    constexpr float r24 = 1.0f / 24.0f;
    const float q = d * r24;
    return __builtin_fmaf(__builtin_fmaf(-q, 24.0f, d), r24, q);
}

// x / c for a float32-valued x and an integer c in [1, 255] with r = fl(1/c):
// q = x*r, remainder fma(-q, c, x) (exact), q' = fma(rem, r, q).  x/c is never a float64
// rounding midpoint and lies >= ulp/(2c) from one, while q' differs from x/c by < 2^-50 ulp,
// so q' is the correctly rounded quotient -- bitwise equal to x / c.  Checked exhaustively for
// every float32 mantissa and every c (tools/check_division.c; scaling by 2^k is exact).
__device__ __forceinline__ double div_by_cap(double x, double c, double r) {
    const double q = x * r;
    return __builtin_fma(__builtin_fma(-q, c, x), r, q);
}

// ---------------------------------------------------------------------------------
// One charger, one step: penalty term of the vehicle present at t-1 and the EV update.
// penalise_charging_vehicles_outside_bounds (penaliser.py:39-57, 71-87): SoC and requested
// SoC at python index t-1.  Charger.charge_or_discharge_vehicle (charger.py:37-56, 58-94,
// 108-144) and reset_info_values (:146-156).
// ---------------------------------------------------------------------------------
struct ChargerResult {
    double pw;      // charger power value (kW), f64 array element of charging_station.py:282
    double q;       // insufficient-charge penalty term (0 if not checked / not insufficient)
    double soc;     // SOC[c, t] after the step
    uint32_t nx;    // 1: non-zero action on an empty charger (100 penalty points, diagnostics only)
    uint32_t fl;
};

// Written with selects rather than branches so the chargers of an env interleave (ILP hides the
// f64 latency at one wavefront per SIMD); the general variant keeps a (divergent) branch for the
// inverted-flag discharge division when dt is not a power of two.  Occupied chargers have cap in [1, 255]
// (validated when a scenario is encoded).
// FAST (NumPy-2 promotion and dt a power of two, e.g. the 1 h default) is straight-line code, so the
// compiler interleaves the chargers of an env.
// NONNEG: the caller knows a >= +0.0 (not NaN, not -0.0): the wide kernel's fast loop, which a wavefront
// takes only when none of its actions is negative, -0.0 or NaN.  Then a vehicle either charges (a > 0) or idles, so the discharge
// branch -- the inverted-flag power (charger.py:122-132) and max(0, calc) -- is never selected and is not
// computed; every value this returns equals the general form's for such actions.
// PK: w is a device-RNG day's packed record (its capacity in bits 3-9), else a word.
template <bool FAST, bool RCP, bool NONNEG = false, bool PK = false>
__device__ __forceinline__ ChargerResult charger_step(const Params &p, uint32_t w, double aux, double run, double req,
                                                      float a, int t, double rcap) {
    ChargerResult o;
    SNG_DIAG_CHARGER(o, aux, run, a);
    const double margin = 0.05 * req;
    const double d = (req - run) * 10;
    const bool insufficient = (t > 0) && (w & W_PEN) && (run < req - margin);
    o.q = insufficient ? d * d : 0.0;

    const bool occ = (w & W_OCC) != 0;
    // previous SoC of an occupied charger, or the recorded SOC[c, t] of an empty one
    const double prev = (occ && !(w & W_STATIC)) ? run : aux;
    const uint32_t capi = cap_field<PK>(w);
    const double cap = (double)capi;
    const bool idle = (a == 0.0f);
    const bool chg = (a > 0.0f);
    double pc, change;
    if (!FAST && p.legacy) {   // NumPy < 2: float32 scalar * int -> float64 (float64 numerator: plain division)
        pc = ((double)a * p.ev_power) * p.ev_eff;
        change = (pc * p.dt) / cap;
    } else {          // NumPy 2 (NEP 50): float32 product
        const float pf = __fmul_rn(__fmul_rn(a, p.ev_power_f), p.ev_eff_f);
        const float pdt = __fmul_rn(pf, p.dt_f);
        pc = (double)pf;
        // RCP: exact reciprocal-fma division with r ~ 1/c (the LDS table, or recip_cap); otherwise
        // the division itself -- all are the IEEE quotient
        change = RCP ? div_by_cap((double)pdt, cap, rcap) : (double)pdt / cap;
    }
    const double calc = prev + change;
    if constexpr (NONNEG) {   // a > 0 charges, a == 0 idles (chg == !idle)
        const bool moved = occ && chg && p.bounded;
        o.soc = moved ? ((1.0 < calc) ? 1.0 : calc) : prev;
        o.pw = moved ? pc : 0.0;
        o.nx = (!occ && chg) ? 1u : 0u;
        o.fl = (occ && chg && !p.bounded) ? (uint32_t)SNG_FLAG_CHARGING_MODE : 0u;
        return o;
    }
    double pw_dis = pc;                                          // inverted flag, charger.py:122-132
    if (FAST) {
        pw_dis = (calc >= 0.0) ? -((prev * cap) * p.rdt) : pc;
    } else if (occ && !idle && !chg && calc >= 0.0) {
        const double x = prev * cap;
        pw_dis = -(p.dt_pow2 ? x * p.rdt : x / p.dt);
    }
    const double soc_chg = (1.0 < calc) ? 1.0 : calc;           // min(calc, 1.0)
    const double soc_dis = (calc > 0.0) ? calc : 0.0;           // max(0.0, calc)
    const bool moved = occ && !idle && p.bounded;
    o.soc = moved ? (chg ? soc_chg : soc_dis) : prev;
    o.pw = moved ? (chg ? pc : pw_dis) : 0.0;                   // full power billed when charging
    o.nx = (!occ && !idle) ? 1u : 0u;
    o.fl = (occ && !idle && !p.bounded) ? (uint32_t)SNG_FLAG_CHARGING_MODE : 0u;
    return o;
}

// ---------------------------------------------------------------------------------
// The BESS step of an env (central_management_system.py:93-94, battery_energy_storage_system.py:30-106,
// penaliser.py:104-111): the new SoC (stored), its penalty and powers, and what it adds to the grid
// balance.  It needs only the BESS SoC and action, not the chargers, so the wide step kernel runs it
// before the charger loop (while the chargers' loads are in flight); env_tail runs it in place otherwise.
// ---------------------------------------------------------------------------------
struct BessStep {
    double bess, pen_b, bpow, bcalc, pw, dp;
    bool moved, chg;
    uint32_t fl;
};
__device__ __forceinline__ BessStep bess_step(const Params &p, const DeviceState &s, uint32_t el8, int t, double bess,
                                              float bess_action) {
    BessStep b{bess, 0.0, 0.0, 0.0, 0.0, 0.0, false, false, 0u};
    if (!p.bess) return b;
    if (t == 0) bst(s.bess0, el8, bess);                       // :93-94
    // charge (ba > 0, battery_energy_storage_system.py:46-74) and discharge (ba < 0, :76-106) share one
    // select-based path with one division: the two branches differ only in their constants, the
    // over-discharge clamp and the SoC bound
    const double ba = (double)bess_action;
    b.chg = ba > 0.0;
    b.pw = (ba * (b.chg ? p.bess_pmax_ch : p.bess_pmax_dis)) * (b.chg ? p.bess_eff_ch : p.bess_eff_dis);
    const double calc = bess + (b.pw * p.dt) / p.bess_cap;
    const double empty = bess * p.bess_cap;   // the over-discharge clamp's energy
    b.dp = (calc < 0.0) ? -(p.dt_pow2 ? empty * p.rdt : empty / p.dt) : b.pw;
    if (ba == 0.0) {
        b.bpow = 0.0;
        b.bcalc = 0.0;
    } else if (!p.bounded) {
        b.fl |= SNG_FLAG_CHARGING_MODE;
    } else {
        b.moved = true;
        b.bcalc = b.pw;
        b.bess = b.chg ? ((1.0 < calc) ? 1.0 : calc) : ((calc > 0.0) ? calc : 0.0);
        b.bpow = b.chg ? b.pw : b.dp;
    }
    if (b.bess < p.bess_dod) {                                 // penaliser.py:104-111
        const double d = (p.bess_dod - b.bess) * 10;
        b.pen_b = d * d;
    } else if (!(b.bess <= 1.0)) {
        b.fl |= SNG_FLAG_BESS_SOC_ABOVE_1;
    }
    bst<kNT>(s.bess, el8, b.bess);
    return b;
}

// ---------------------------------------------------------------------------------
// Env tail: BESS (unless PRE: bess_step ran before the chargers), grid energy, cost, reward
// (central_management_system.py:99-185, penaliser.py:177-187, accountant.py:26-40) and the observation's
// BESS entry.  Leader lane only.
// ---------------------------------------------------------------------------------
static_assert((SNG_FLAG_NEGATIVE_DEMAND | SNG_FLAG_CHARGING_MODE | SNG_FLAG_BESS_SOC_ABOVE_1 | SNG_FLAG_V2X_BREAKPOINT) == 0xfu,
              "env_tail ORs the flag summary bit by bit: bits 0-3");
template <bool DIAG, bool PRE = false>
__device__ __forceinline__ void env_tail(const Params &p, const DeviceState &s, const InfoPtrs &info, int64_t e0, uint32_t lo, uint32_t el1, uint32_t el8,
                                         int t, double ratio, double bess, float bess_action, double p_ch,
                                         double p_dis, double pen_v, double nonexist, uint32_t fl, float *o_row,
                                         const double *cst, const double *fpv, const double *fpr, double ret_prev,
                                         double bess0, double *__restrict__ reward, uint8_t *__restrict__ done,
                                         const BessStep *pre = nullptr) {
    // no global loads in here: a load would wait (vmcnt) for every SoC store the env just issued
    const double solar = p.pv ? (cst[CST_PV] * ratio) * fpv[0] : 0.0;   // central_management_system.py:99-103
    const double demand = p_ch + p_dis;                            // :105
    if (demand < 0.0) fl |= p.v2x ? SNG_FLAG_V2X_BREAKPOINT : SNG_FLAG_NEGATIVE_DEMAND;
    double rem = demand - solar;                                   // :167

    if (p.bess && t == 0) bess0 = bess;
    const BessStep b = PRE ? *pre : bess_step(p, s, el8, t, bess, bess_action);
    fl |= b.fl;
    if (b.moved) rem = b.chg ? -((-rem) - b.pw) : rem + b.dp;     // battery_energy_storage_system.py:46-106
    const double pen_b = b.pen_b, bpow = b.bpow, bcalc = b.bcalc;
    bess = b.bess;

    const double grid = rem;
    const double energy = grid * p.dt;
    const double price = cst[CST_PRICE] * fpr[0];
    const double cost = (energy < 0.0) ? (energy * p.sell_coef) * price : energy * price;
    const double tot_pen = p.bat_pen_w * pen_b + pen_v;
    const double total = p.grid_w * fabs(cost) + tot_pen;
    bst<kNT>(reward, el8, -total);
    bst<kNT>(done, el1, (uint8_t)((t + 1 == p.T) ? 1 : 0));

    // (the observation header was written before the chargers: step_kernel)
    if (p.bess && !PRE) o_row[p.obs_dim - 1] = (float)bess;

    if (fl) atomicOr(s.flags + e0 + lo, fl);   // sticky per-env error bits; no-return atomics, nothing waits
    // the flag summary (SngInfo.flag_summary): the wavefront's active lanes' bits ORed by one ballot per flag
    // bit (four: sng.h), then one atomic per wavefront into the wavefront's own word.  A V2X station flags
    // most envs on most steps: one atomic per flagged env into one shared word cost 18.9 us per
    // step at N = 10, one per wavefront into that word 17.6 us -- the device-scope atomics on one address run
    // one after another at the memory side, and the last wavefronts waited ~10 us for theirs
    // (profiles/r05_stamps_v2x.txt) -- and one per wavefront into its own word 7.1 us.  A wavefront without a
    // flag pays one ballot.
    if (info.flag_any && __builtin_amdgcn_ballot_w64(fl != 0u)) {
        uint32_t any = 0u;
#pragma unroll
        for (uint32_t b = 1u; b <= SNG_FLAG_V2X_BREAKPOINT; b <<= 1)
            any |= __builtin_amdgcn_ballot_w64((fl & b) != 0u) ? b : 0u;
        if (__lane_id() == (unsigned)__builtin_ctzll(__builtin_amdgcn_read_exec()))
            atomicOr(info.flag_any + ((uint32_t)(e0 >> 5) & (SNG_FLAG_SUMMARY_WORDS - 1)), any);
    }
    if (info.flags) bst(info.flags, el1 * 4u, fl);
    if (info.episode_return) bst<kNT>(info.episode_return, el8, ret_prev + -total);
    if (DIAG) {
        if (info.grid_power) bst(info.grid_power, el8, (double)(grid));
        if (info.p_charge) bst(info.p_charge, el8, (double)(p_ch));
        if (info.p_discharge) bst(info.p_discharge, el8, (double)(p_dis));
        if (info.bess_soc) bst(info.bess_soc, el8, (double)(p.bess ? bess : 0.0));
        if (info.pen_vehicle) bst(info.pen_vehicle, el8, (double)(pen_v));
        if (info.pen_battery) bst(info.pen_battery, el8, (double)(pen_b));
        if (info.grid_cost) bst(info.grid_cost, el8, (double)(cost));
        if (info.total_cost) bst(info.total_cost, el8, (double)(total));
        if (info.solar) bst(info.solar, el8, (double)(solar));
        if (info.bess_power) bst(info.bess_power, el8, (double)(bpow));
        if (info.bess_calc_power) bst(info.bess_calc_power, el8, (double)(bcalc));
        if (info.nonexistent) bst(info.nonexistent, el8, (double)(nonexist));
        if (info.bess_initial) bst(info.bess_initial, el8, (double)(p.bess ? bess0 : 0.0));
    }
}

// Workgroup size of the step kernel: 256 threads (4 wavefronts, 4x fewer workgroups to
// dispatch) while the LDS staging fits, one wavefront for wide stations (N > 16 or runtime N)
// so the [ENVS][O] observation tile stays well inside the 160 KB LDS.
__host__ __device__ constexpr int step_block(int NC) { return (NC > 0 && NC <= 16) ? 256 : 64; }

// LDS carve-up of the step kernel, one slice per wavefront (every region 16-byte aligned):
//   act [WENVS][A] f32 | obs [WENVS][O] f32 | (kRows) rcp [256] f64 | (kRows) cst [16] f64
//   | pos [WENVS][NC] f64 | neg [WENVS][NC] f64 | (L > 1) pw [WENVS][NC] f64
// With L > 1 the penalty rows q [WENVS][NC] f64 share the first region with the actions tile:
// a lane's chargers are one batch, whose action reads all precede the first q write in the
// wavefront's program order (the BESS action is read before the loop).
// Each wavefront stages, computes and writes back its own 64/L envs: no workgroup barrier, so
// the waves of a CU drift apart and one wave's loads overlap another's arithmetic and stores.
template <int NC, int L>
struct StepLds {
    static constexpr int BLOCK = step_block(NC);
    static constexpr int WAVES = BLOCK / kWave;
    static constexpr int WENVS = kWave / L;              // envs per wavefront
    static constexpr int ENVS = WAVES * WENVS;           // envs per workgroup
    static constexpr bool kRows = NC > 0 && NC <= 16;   // compacted power rows (else PairwiseSum)
    __host__ __device__ static int act_floats(int A) { return round4(WENVS * A); }
    __host__ __device__ static int obs_floats(int O) { return round4(WENVS * O); }
    // wide stations (!kRows) keep no 1/c table and no step constants in LDS: at N = 50 the act
    // and obs tiles alone are 40 KB per wavefront, and 40 KB is what lets 4 wavefronts (one per
    // SIMD) share a CU's 160 KB
    __host__ __device__ static size_t first_bytes(int A) {   // actions tile, or the q rows aliasing it
        const size_t a = (size_t)act_floats(A) * 4, q = L > 1 ? (size_t)WENVS * NC * 8 : 0;
        return a > q ? a : q;
    }
    __host__ __device__ static size_t wave_bytes(int A, int O) {
        size_t b = first_bytes(A) + (size_t)obs_floats(O) * 4;
        if (kRows) b += (size_t)(256 + 16) * 8 + (size_t)2 * WENVS * NC * 8;
        if (L > 1) b += (size_t)WENVS * NC * 8;
        return b;
    }
    __host__ __device__ static size_t bytes(int A, int O) { return WAVES * wave_bytes(A, O); }
};

// Chargers per batch of the one-lane step kernel: all of them up to 16; for wider stations the
// largest divisor of N in [10, 16] (no ragged last batch), else 8 -- each batch's loads are issued
// together and then consumed.  Measured at N = 50 (config 5): batches of 10 33.1 us per step, 17
// 33.5, 25 34.5, 13 36.8, 8 39.1.
__host__ __device__ constexpr int wide_batch(int NC) {
    if (NC > 0 && NC <= 16) return NC;
    for (int d = 16; d >= 10; --d)
        if (NC > 0 && NC % d == 0) return d;
    return 8;
}

// LDS ordering inside one wavefront: a wave's LDS operations complete in issue order, so a
// compiler-level fence is all that is needed between the writes of some lanes and the reads of
// others (no s_barrier).
__device__ __forceinline__ void wave_lds_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 1/c for an integer capacity c in [1, 255]: v_rcp_f64 and one Newton step.  div_by_cap needs only a
// relative error far below 2^-31 here (its quotient then errs by < 2^-62 relative before the last
// rounding, which x/c's distance from a rounding midpoint, >= 2^-62, absorbs): v_rcp_f64's error
// squared by the Newton step is ~2^-46.  c = 0 (empty charger) gives NaN, which charger_step selects away.
__device__ __forceinline__ double recip_cap(double c) {
    const double r0 = __builtin_amdgcn_rcp(c);
    return __builtin_fma(r0, __builtin_fma(-c, r0, 1.0), r0);
}

// ---------------------------------------------------------------------------------
// The lean step kernel: the one-lane, no-diagnostics, NumPy-2 / power-of-two-dt step of a station of
// N <= 16 chargers without stochastic profiles (every configuration the bench and a training loop
// run), one wavefront per 64 envs, 4 wavefronts per workgroup with wavefront-private LDS tiles.
// Against the general step_kernel below:
//   - the prologue is one kernarg round trip: no early exit (a wavefront past E loads env E - 1 and
//     stores nothing), no runtime branch before the loads (the requested-SoC stream is the template
//     argument REQ), and this step's table constants arrive by value (StepConst) instead of through
//     the tables pointer, so every vector load issues right after the kernel arguments land;
//   - nothing but the actions and observation tiles lives in LDS: 1/cap comes from recip_cap (no
//     per-wavefront table staging, no LDS round trip per charger);
//   - the charging / discharging totals are the running sums the lane keeps anyway whenever those
//     equal numpy's pairwise sum of the compacted arrays (charging_station.py:289-293) exactly:
//       * fewer than 8 terms: numpy sums them sequentially (loops_utils.h.src), and the skipped +0.0
//         terms leave a sum unchanged;
//       * positive powers are float32 values (the NEP 50 product pc, charger.py:92-94, when
//         charging); when the smallest of them, pmin, satisfies sum <= pmin * 2^28, every partial sum
//         is a multiple of pmin's float32 ulp below 2^53 such ulps, so every addition is exact in any
//         order.
//     Only a lane with 8 or more negative powers, or 8 or more positive ones whose sum is not
//     provably exact, compacts its powers into its LDS rows and runs the pairwise sum (rare; skipped
//     wave-uniformly otherwise).
// ---------------------------------------------------------------------------------
struct StepConst {
    double v[CST_COUNT];   // step_constant(tables, t, i) for i < CST_COUNT
};

// Threads per workgroup of the lean step kernel: one wavefront (1,024 workgroups at E = 65,536).
// A/B on one box (day of 65,536 x 10): 64 threads 6.33-6.38 us per step, 256 threads 6.47-6.55,
// 128 threads 7.13-7.14 (library A/B: tools/diag/variant.sh builds, tools/gpu_session.sh ablib runs them).
constexpr int kLeanBlock = 64;

template <int NC>
struct LeanLds {
    static constexpr int A = NC + 1;   // actions per env with a BESS (one fewer without)
    static constexpr int O = 2 * NC + 9;
    static constexpr int ACT = round4(kWave * A), OBS = round4(kWave * O);
    static constexpr size_t WAVE_BYTES = (size_t)(ACT + OBS) * 4 + (size_t)2 * kWave * NC * 8;
    static constexpr size_t BYTES = (kLeanBlock / kWave) * WAVE_BYTES;
};

template <int NC, bool PK, bool REQ>
__global__ __launch_bounds__(kLeanBlock) void step_lean_kernel(const float *__restrict__ act, float *__restrict__ obs,
                                                        double *__restrict__ reward, uint8_t *__restrict__ done,
                                                        int64_t E, int t, int vec_io, StepConst k, Params p,
                                                        DeviceState s, InfoPtrs info) {
    using Lay = LeanLds<NC>;
    constexpr int KT = (Lay::A * kWave + 4 * kWave - 1) / (4 * kWave);
    extern __shared__ __attribute__((aligned(16))) float lds[];
    SNG_WSTAMP_DECL;
    SNG_WSTAMP(0);
    const int Ad = p.act_dim, O = p.obs_dim;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int64_t e0 = (int64_t)blockIdx.x * kLeanBlock + (int64_t)wave * kWave;
    const int64_t rem_e = E - e0;
    const int nw = rem_e <= 0 ? 0 : (rem_e < kWave ? (int)rem_e : kWave);
    const bool live = lane < nw;
    float *s_act = reinterpret_cast<float *>(reinterpret_cast<char *>(lds) + wave * Lay::WAVE_BYTES);
    float *s_obs = s_act + Lay::ACT;
    double *s_pos = reinterpret_cast<double *>(s_obs + Lay::OBS);
    double *s_neg = s_pos + kWave * NC;
    const int64_t el = live ? e0 + lane : E - 1;   // idle lanes load a valid env and discard it
    const int64_t ew = nw > 0 ? e0 : E - 1;         // a wavefront past E stages env E - 1's row
    const uint32_t el1 = (uint32_t)el, el4 = el1 * 4u, el8 = el1 * 8u;
    const size_t plane = (size_t)t * NC * (size_t)E;   // this step's timeline planes

    // loads oldest-needed-first, all behind the one kernarg wait: the wave's actions tile and the
    // per-env values (the LDS commit and the observation header wait for them, before any charger),
    // then the per-charger state, which charger c waits for in order
    TileStage<KT, kWave> act_tile;
    act_tile.issue(act + ew * Ad, (nw > 0 ? nw : 1) * Ad, vec_io != 0, lane);
    const double ratio = bld(s.ratio, el8);   // pointer selects rather than branches: a disabled
    const double bess_l = bld(p.bess ? s.bess : s.ratio, el8);   // stream re-reads ratio
    const double pen0_l = bld(t == 0 ? s.pen0 : s.ratio, el8);
    const double ret_l = bld(info.episode_return ? info.episode_return : s.ratio, el8);
    uint32_t w[NC];
    double aux[NC], run[NC], req[NC];
    const uint16_t *rec_t = packed_records(s) + plane + (size_t)NC * (size_t)E;   // t + 1
#pragma unroll
    for (int c0 = 0; c0 < NC; c0 += 2) {   // charger pairs: the SoC state's 16 B slots (sng_layout.h)
        if (PK && (c0 & 3) == 0) {   // packed device-day records (sng_layout.h), plane t + 1: a quad per 8 B
            if (c0 + 4 <= NC) {
                unpack_quad(bld(reinterpret_cast<const uint64_t *>(rec_t), el1 * 8u, (uint32_t)c0 * (uint32_t)E * 2u), w + c0);
            } else {
#pragma unroll
                for (int c = c0; c < NC; ++c) {
                    const RecOff ro = rec_off(c, NC, E, el1);
                    w[c] = bld16(rec_t, ro.v, ro.s);
                }
            }
        }
#pragma unroll
        for (int c = c0; c < c0 + 2 && c < NC; ++c) {
            const uint32_t r4 = (uint32_t)c * (uint32_t)E * 4u, r8 = 2u * r4;   // charger row
            if (!PK) {
                w[c] = bld(s.word + plane, el4, r4);
                aux[c] = bld(s.aux + plane, el8, r8);
            }
        }
        if (c0 + 1 < NC)
            bld2(s.soc, 2u * el8, (uint32_t)c0 * (uint32_t)E * 8u, run[c0], run[c0 + 1]);
        else
            run[c0] = bld(s.soc, el8, (uint32_t)c0 * (uint32_t)E * 8u);
        // Requested_SOC[c, t-1]; without the stream 1.0 (charging_station.py:230-232), or the cleared
        // 0.0 of a replayed day (Params::req_zero)
#pragma unroll
        for (int c = c0; c < c0 + 2 && c < NC; ++c)
            req[c] = REQ ? bld(s.req + plane, el8, (uint32_t)c * (uint32_t)E * 8u) : (p.req_zero ? 0.0 : 1.0);
    }
    act_tile.commit(s_act, lane);
    wave_lds_fence();
    SNG_WSTAMP(1);

    const float *a_row = s_act + lane * Ad;
    float *o_row = s_obs + lane * O;
    float av[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) av[c] = a_row[c];
    const float bess_action = p.bess ? a_row[NC] : 0.0f;
    const int k_soc = p.pv ? 8 : 4;
    const double one4[4] = {1.0, 1.0, 1.0, 1.0};
    // the header needs only the PV ratio and the constants: written while the chargers' loads fly
    if (live) write_obs_header(o_row, p, k.v + CST_IRR, k.v + CST_PN, ratio, one4, one4);

    double pwv[NC], sv[NC];
    double pen_v = 0.0, seq_pos = 0.0, seq_neg = 0.0, pmin = __builtin_inf();
    int n_pos = 0, n_neg = 0;
    uint32_t n_nonexist = 0, fl = 0;
    bool pos_other = false;   // a positive power that is not the float32 charging product
    if (live) {
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const uint32_t capi = cap_field<PK>(w[c]);
            // a packed day: an arriving vehicle's SoC is the running SoC the step before stored (the
            // record it carried), so the step sees no STATIC bit and an empty charger's SoC is 0
            const bool occ = (w[c] & W_OCC) != 0;
            const ChargerResult r = charger_step<true, true, false, PK>(p, PK ? (w[c] & ~W_STATIC) : w[c], PK ? 0.0 : aux[c],
                                                                        run[c], req[c], av[c], t, recip_cap((double)capi));
            sv[c] = (PK && !occ) ? (double)rec_soc(w[c]) : r.soc;
            if (c & 1)   // the pair's 16 B slot once both chargers are stepped
                bst2<kNT>(s.soc, 2u * el8, sv[c - 1], sv[c], (uint32_t)(c - 1) * (uint32_t)E * 8u);
            else if (c == NC - 1)
                bst<kNT>(s.soc, el8, sv[c], (uint32_t)c * (uint32_t)E * 8u);
            o_row[k_soc + c] = (float)r.soc;
            o_row[k_soc + NC + c] = departure_obs<PK>((PK && !occ) ? 0u : w[c]);
            n_nonexist += r.nx;
            fl |= r.fl;
            pen_v += r.q;
            const double pw = r.pw;
            pwv[c] = pw;
            const bool ip = pw > 0.0;
            seq_pos += __builtin_fmax(pw, 0.0);   // v_max/v_min drop a NaN power, as P[P > 0] does
            seq_neg += __builtin_fmin(pw, 0.0);
            n_pos += ip ? 1 : 0;
            n_neg += (pw < 0.0) ? 1 : 0;
            pmin = __builtin_fmin(pmin, ip ? pw : __builtin_inf());
            pos_other |= ip && !(av[c] > 0.0f);
            // chargers in order: charger c waits only for its own loads (vmcnt counts down charger
            // by charger) while the later chargers' loads are in flight
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    SNG_WSTAMP(2);
    double p_ch = seq_pos, p_dis = seq_neg;
    if constexpr (NC >= 8) {
        const bool pos_slow = n_pos >= 8 && (pos_other || !(seq_pos <= pmin * 0x1.0p28));
        const bool slow = live && (pos_slow || n_neg >= 8);
        if (__builtin_amdgcn_ballot_w64(slow)) {   // wave-uniform: rare
            if (slow) {
                double *row_pos = s_pos + lane * NC, *row_neg = s_neg + lane * NC;
                int kp = 0, kn = 0;
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    row_pos[kp] = pwv[c];
                    row_neg[kn] = pwv[c];
                    kp += (pwv[c] > 0.0) ? 1 : 0;
                    kn += (pwv[c] < 0.0) ? 1 : 0;
                }
                p_ch = pairwise_row_c<NC>(row_pos, n_pos, seq_pos);
                p_dis = pairwise_row_c<NC>(row_neg, n_neg, seq_neg);
            }
        }
    }
    if (live) {
        // t = 0 reads the python index -1 slot (pen0); the per-charger terms are all 0 there
        pen_v += (t == 0) ? pen0_l : 0.0;
        env_tail<false>(p, s, info, e0, (uint32_t)lane, el1, el8, t, ratio, p.bess ? bess_l : 0.0, bess_action,
                        p_ch, p_dis, pen_v, 100.0 * (double)n_nonexist, fl, o_row, k.v, one4, one4,
                        info.episode_return ? ret_l : 0.0, 0.0, reward, done);
    }
    wave_lds_fence();
    SNG_WSTAMP(3);
    if (nw > 0) copy_out<kWave>(obs + e0 * O, s_obs, nw * O, vec_io != 0, lane);
    SNG_WSTAMP(4);
    SNG_WSTAMP_FLUSH(stamp_, 5);
    // a device-RNG day's first step advances the day counter its reset read (generate_kernel); no-return
    // atomic, so nothing waits for it.  A replayed day (bump_day = 0) drew no counter value of its own.
    if (PK && t == 0 && p.bump_day && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_add(s.episode, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------
// The wide lean step kernel: step_lean_kernel's recipe for stations wider than 16 chargers (BASELINE
// config 5: N = 50, 15-minute steps, stochastic PV / price profiles), one wavefront per 64 envs, one
// wavefront per workgroup, one wavefront per SIMD at E = 65,536 (so the whole 512-entry register file:
// every charger's state is loaded up front).  What makes it lean at N = 50:
//   - the charging total is the running sum whenever that equals numpy's pairwise sum of the compacted
//     positive powers exactly (step_lean_kernel's argument: fewer than 8 terms, or float32 powers whose
//     sum stays below 2^28 times the smallest), instead of numpy's 8-accumulator schedule fed one
//     power at a time (PairwiseSum: ~40 VALU per power, two per charger);
//   - the discharging total is exactly 0.0 (numpy's sum of an empty array) when no action of the wave is
//     negative: a negative power needs a negative action (charger.py:37-56, 108-140), and then no power
//     is positive other than a charging product.  A wavefront with a negative action (V2X) takes the
//     general order, PairwiseSum over both signs, in a rolled loop that re-reads each charger's inputs
//     (rare: nothing in the fast loop indexes the register arrays at run time);
//   - a lane whose positive sum is not provably exact rebuilds its compacted positive powers from what
//     the step leaves unchanged -- the records (occupancy) and the actions tile (the float32 product
//     charger.py:92-94) -- and sums them in numpy's order (rare);
//   - constants by value, one kernarg round trip before the loads, 1/cap by recip_cap, no LDS but the
//     actions and observation tiles (40 KB per wavefront: four per CU).
// ---------------------------------------------------------------------------------

template <int NC, int L>
struct WideLds {
    static constexpr int WENVS = kWave / L;   // envs per wavefront
    static constexpr int A = NC + 1;          // actions per env with a BESS (one fewer without)
    static constexpr int O = 2 * NC + 9;
    static constexpr int ACT = round4(WENVS * A), OBS = round4(WENVS * O);
    static constexpr size_t BYTES = (size_t)(ACT + OBS) * 4;
};

// The NEP 50 float32 charging power of action a (charger.py:92-94), as charger_step computes it.
__device__ __forceinline__ double charging_power(const Params &p, float a) {
    return (double)__fmul_rn(__fmul_rn(a, p.ev_power_f), p.ev_eff_f);
}

// Lane `part` K's value of an env's L adjacent lanes (L = 2 or 4), for the env's first lane, by DPP quad
// permutation (the env's lanes never straddle a quad).
template <int L, int K>
__device__ __forceinline__ uint32_t from_part(uint32_t x) {
    constexpr int ctrl = L == 2 ? (K | (K << 2) | ((K + 2) << 4) | ((K + 2) << 6)) : (K | (K << 2) | (K << 4) | (K << 6));
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, ctrl, 0xF, 0xF, false);
}
template <int L, int K>
__device__ __forceinline__ double from_part(double x) {
    const uint64_t b = __builtin_bit_cast(uint64_t, x);
    const uint64_t lo = from_part<L, K>((uint32_t)b), hi = from_part<L, K>((uint32_t)(b >> 32));
    return __builtin_bit_cast(double, lo | (hi << 32));
}

// L lanes per env (1, 2 or 4): lane `part` of an env steps chargers [part * CPL, min(NC, (part + 1) * CPL)),
// CPL = ceil(NC / L).  The env's lanes are adjacent (one DPP quad); the partial charging sums, counts and
// minima combine exactly on the first lane (a sum the exactness test accepts is exact in any order, and
// fewer than 8 powers are numpy's in-order sum when one lane holds them all), the first lane adds the
// other lanes' vehicle penalties after its own in charger order (Python's sum, penaliser.py:55), and the
// rare exact-order paths run on the first lane over all chargers.
// One group of WENVS envs of a wavefront: its loads (issue), then its step (run).  A wavefront steps G
// groups: every group's loads are issued before the first group is stepped, so a group's arithmetic and
// stores overlap the later groups' loads still in flight (G = 1: the whole wavefront is one group).
template <int NC, int L, bool PK, bool REQ, bool NOISE>
struct WideGroup {
    using Lay = WideLds<NC, L>;
    static constexpr int WENVS = Lay::WENVS, CPL = (NC + L - 1) / L;
    static constexpr int KT = (Lay::A * WENVS + 4 * kWave - 1) / (4 * kWave);
    static_assert((L - 1) * CPL < NC, "every lane steps at least one charger");
    // The lane's chargers.  Two lanes and N = 2 mod 4 (the headline's 10, config 5's 50): lane `part` steps the
    // whole charger pairs [part H, part H + H) (H = (N - 2) / 2) and charger N - 2 + part of the last pair, so
    // its SoC state moves as 16 B charger pairs (sng_layout.h) but for that last charger.  Otherwise the
    // contiguous ranges [part CPL, min(N, part CPL + CPL)).
    static constexpr bool kPairs = L == 2 && NC % 4 == 2;
    // the fast loop's charger step without the discharge branch (charger_step NONNEG) for the headline's
    // station (step 6.60-6.66 -> 6.53-6.56 us, profiles/r04_ab_nonneg.txt).  At N = 50 the compiler merges
    // several chargers' select masks ahead of the per-charger scheduling barriers and spills them (332
    // v_readlane); with each charger's inputs pinned to its block it compiles to 5.5 % fewer VALU, and
    // config 5 ran 22.62-22.69 against 22.47-22.54 us (profiles/r04_ab_config5_nonneg.txt): its step is
    // bound by its bytes, so config 5 keeps the general form
    static constexpr bool kNonneg = NC <= 16;
    static constexpr int H = (NC - 2) / 2;
    static_assert(!kPairs || CPL == H + 1, "a lane's chargers: H from whole pairs and one from the last");
    // the lane's whole pairs are whole record quads too (H a multiple of 4: N = 10, 50), and the last pair is
    // the partial quad's two records
    static constexpr bool kQuads = kPairs && H % 4 == 0;
    static __device__ __forceinline__ int charger(int part, int j) {
        return kPairs ? (j < H ? part * H + j : NC - 2 + part) : part * CPL + j;
    }
    int64_t e0;
    int nw;
    bool live;
    uint32_t el1, el4, el8, row4, row4_last, soc_a, soc_b, rec_a, rec_b;
    TileStage<KT, kWave> act_tile;
    double ratio, bess_l, pen0_l, ret_l;
    double fpv[4], fpr[4];
    uint32_t w[CPL];
    double aux[PK ? 1 : CPL], run_[CPL], req[REQ ? CPL : 1];
    SNG_WSTAMP_DECL;   // diagnostic builds: 0 issue, 1 actions tile staged, 2 chargers, 3 env tail, 4 obs stores issued

    // the (per-lane, uniform) byte offsets of charger j of the lane in a [N][E] u32 plane: j * E in the uniform
    // part, except for the j some lane lacks (a ragged last lane) or the last pair's charger, where the
    // per-lane part carries it
    static __device__ __forceinline__ bool ragged(int j) { return !kPairs && NC % L != 0 && j >= NC - (L - 1) * CPL; }
    __device__ __forceinline__ uint32_t r4_of(int j, int64_t E) const {
        if constexpr (kPairs) return (uint32_t)(j < H ? j : NC - 2) * (uint32_t)E * 4u;
        return ragged(j) ? 0u : (uint32_t)j * (uint32_t)E * 4u;
    }
    __device__ __forceinline__ uint32_t row_of(int j, int nc, int64_t E) const {
        if constexpr (kPairs) return j < H ? row4 : row4_last;
        return ragged(j) ? (j < nc ? row4 + (uint32_t)j * (uint32_t)E * 4u : row4_last) : row4;
    }
    // loads oldest-needed-first: the actions tile and the per-env values, then every charger's state
    __device__ __forceinline__ void issue(int64_t e0_, const float *act, int64_t E, int t, int vec_io, const Params &p,
                                          const DeviceState &s, const InfoPtrs &info, int lane) {
        SNG_WSTAMP(0);
        const int le = lane / L, part = lane % L;
        e0 = e0_;
        nw = (E - e0) < WENVS ? (int)(E - e0) : WENVS;
        live = le < nw;
        const int64_t el = live ? e0 + le : E - 1;   // idle lanes load a valid env and discard it
        el1 = (uint32_t)el;
        el4 = el1 * 4u;
        el8 = el1 * 8u;
        const int c0 = part * CPL;
        const int nc = kPairs ? CPL : ((NC - c0) < CPL ? NC - c0 : CPL);
        if constexpr (kPairs) {
            row4 = el4 + (uint32_t)(part * H) * (uint32_t)E * 4u;     // charger part H + j, j < H: + j E (uniform)
            row4_last = el4 + (uint32_t)part * (uint32_t)E * 4u;      // charger N - 2 + part: + (N - 2) E (uniform)
            soc_a = 2u * el8 + (uint32_t)(part * H) * (uint32_t)E * 8u;   // pair row part H + j: + j E 8 (uniform)
            soc_b = 2u * el8 + (uint32_t)part * 8u;                      // the last pair's row: + (N - 2) E 8
            rec_a = el1 * 8u + (uint32_t)(part * H) * (uint32_t)E * 2u;   // quad row part H + j: + j E 2 (uniform)
            rec_b = el1 * 4u + (uint32_t)part * 2u;                      // the partial quad (N - 2, N - 1): + (N - 2) E 2
        } else {
            // the lane's first charger row as a per-lane byte offset; charger j of the lane adds j * E
            // (uniform).  Past the lane's range (j >= nc) the loads re-read its first charger and nothing is
            // stored.
            row4 = el4 + (uint32_t)c0 * (uint32_t)E * 4u;
            row4_last = el4 + (uint32_t)(NC - 1) * (uint32_t)E * 4u;
        }
        const size_t plane = (size_t)t * NC * (size_t)E;   // this step's timeline planes
        const uint16_t *rec_t = packed_records(s) + plane + (size_t)NC * (size_t)E;   // t + 1
        const int Ad = p.act_dim;
        act_tile.issue(act + e0 * Ad, nw * Ad, vec_io != 0, lane);
        ratio = bld(s.ratio, el8);
        bess_l = bld(p.bess ? s.bess : s.ratio, el8);
#pragma unroll
        for (int j = 0; j < 4; ++j) fpv[j] = fpr[j] = 1.0;
        if constexpr (NOISE) profile_factors(p, s, el8, t, fpv, fpr);   // the day's profile factors of t..t+3
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            // charger `charger(part, j)` (past a ragged lane's range: its charger NC - 1 again, discarded)
            const uint32_t v4 = row_of(j, nc, E), r4 = r4_of(j, E), v8 = 2u * v4, r8 = 2u * r4;
            if (PK) {   // 2 B records in charger quads: the lane's whole quads as 8 B, its last-pair charger as 2 B
                if constexpr (kQuads) {
                    if (j < H && (j & 3) == 0)
                        unpack_quad(bld(reinterpret_cast<const uint64_t *>(rec_t), rec_a, (uint32_t)j * (uint32_t)E * 2u),
                                    w + j);
                    if (j == H) w[j] = bld16(rec_t, rec_b, (uint32_t)(NC - 2) * (uint32_t)E * 2u);
                } else {
                    const int cr = charger(part, j) < NC ? charger(part, j) : NC - 1;
                    const RecOff ro = rec_off(cr, NC, E, el1);
                    w[j] = bld16(rec_t, ro.v, ro.s);
                }
            } else {
                w[j] = bld(s.word + plane, v4, r4);
                aux[PK ? 0 : j] = bld(s.aux + plane, v8, r8);
            }
            if constexpr (kPairs) {   // a pair's 16 B once both its records are issued; the last pair's 8 B
                if (j < H && (j & 1)) bld2(s.soc, soc_a, (uint32_t)(j - 1) * (uint32_t)E * 8u, run_[j - 1], run_[j]);
                if (j == H) run_[j] = bld(s.soc, soc_b, (uint32_t)(NC - 2) * (uint32_t)E * 8u);
            } else {
                const int c = c0 + j < NC ? c0 + j : NC - 1;
                run_[j] = bld(s.soc, (uint32_t)soc_index(c, el, NC, E) * 8u);
            }
            if (REQ) req[REQ ? j : 0] = bld(s.req + plane, v8, r8);
        }
        // the t = 0 penalty and the day return are read only by the env tail: issued behind every charger's
        // loads, so the waits before the chargers (the header's PV ratio, the BESS step's SoC) do not count them
        // (round 6, A/B in the day graph: 6.36 -> 6.25-6.29 us per step, profiles/r06_ab_step_tail_order.txt).
        // Stores issued earlier or in bursts measured slower there: the observation tile stored before the env
        // tail +0.33 us, its copy-out unrolled (every LDS read, then every 16 B store) +0.6 us, the SoC pairs
        // stored after the charger loop +0.3 us -- paced stores leave the other wavefronts' loads alone.
        pen0_l = bld(t == 0 ? s.pen0 : s.ratio, el8);
        ret_l = bld(info.episode_return ? info.episode_return : s.ratio, el8);
    }
    // Requested_SOC[c, t-1] of charger j of the lane; without the stream 1.0, or the cleared 0.0 of a replayed day
    __device__ __forceinline__ double req_of(int j, const Params &p) const {
        return REQ ? req[REQ ? j : 0] : (p.req_zero ? 0.0 : 1.0);
    }

    // the group's step; s_act holds its actions tile (committed), s_obs is the wavefront's observation tile
    __device__ __forceinline__ void run(const float *s_act, float *s_obs, float *obs, double *reward, uint8_t *done,
                                        int64_t E, int t, int vec_io, const StepConst &k, const Params &p,
                                        const DeviceState &s, const InfoPtrs &info, int lane) {
        SNG_WSTAMP(1);
        const int Ad = p.act_dim, O = p.obs_dim;
        const int le = lane / L, part = lane % L;
        const bool leader = part == 0;
        const int c0 = part * CPL;
        const int nc = kPairs ? CPL : ((NC - c0) < CPL ? NC - c0 : CPL);
        const size_t plane = (size_t)t * NC * (size_t)E;
        const uint16_t *rec_t = packed_records(s) + plane + (size_t)NC * (size_t)E;
        const float *a_row = s_act + le * Ad;
        float *o_row = s_obs + le * O;
        float av[CPL];
        // the largest action bit pattern: above +inf's (0x7f800000) when some action is negative (-0.0 too) or
        // NaN, and such a wavefront takes the general order below (an integer max keeps no per-charger lane
        // masks alive into the charger loop)
        uint32_t amax_bits = 0u;
#pragma unroll
        for (int j = 0; j < CPL; ++j) {
            const int c = charger(part, j);
            av[j] = a_row[c < NC ? c : NC - 1];
            amax_bits = __builtin_elementwise_max(amax_bits, __builtin_bit_cast(uint32_t, av[j]));
        }
        const bool not_nonneg = amax_bits > 0x7f800000u;
        const float bess_action = p.bess ? a_row[NC] : 0.0f;
        const int k_soc = p.pv ? 8 : 4;
        // the observation header and the BESS step need only per-env values: both run here, while the
        // chargers' loads are still in flight (the BESS's division no longer trails the charger sums)
        BessStep bs{};
        if (live && leader) {
            write_obs_header(o_row, p, k.v + CST_IRR, k.v + CST_PN, ratio, fpv, fpr);
            bs = bess_step(p, s, el8, t, p.bess ? bess_l : 0.0, bess_action);
            if (p.bess) o_row[O - 1] = (float)bs.bess;
        }

        double pen_v = 0.0, p_ch = 0.0, p_dis = 0.0;
        uint32_t n_nonexist = 0, fl = 0;
        if (__builtin_amdgcn_ballot_w64(live && not_nonneg) == 0) {
            // the fast loop: every action of the wave is >= 0, so no negative power (p_dis stays 0.0) and no
            // charger discharges (charger_step<..., NONNEG>)
            double seq_pos = 0.0, pmin = __builtin_inf();
            int n_pos = 0;
            double qv[L > 1 ? CPL : 1], sv[CPL];
            if (live) {
#pragma unroll
                for (int j = 0; j < CPL; ++j) {
                    const int c = charger(part, j);
                    if (!kPairs && NC % L != 0 && j >= nc) {   // a ragged lane's range ends: adds nothing
                        qv[L > 1 ? j : 0] = 0.0;
                        continue;
                    }
                    const uint32_t capi = cap_field<PK>(w[j]);
                    const bool occ = (w[j] & W_OCC) != 0;
                    const ChargerResult r = charger_step<true, true, kNonneg, PK>(p, PK ? (w[j] & ~W_STATIC) : w[j],
                                                                           PK ? 0.0 : aux[PK ? 0 : j], run_[j], req_of(j, p),
                                                                           av[j], t, recip_cap((double)capi));
                    sv[j] = (PK && !occ) ? (double)rec_soc(w[j]) : r.soc;
                    if constexpr (kPairs) {   // a pair's 16 B once both its chargers are stepped; the last pair's 8 B
                        if (j < H && (j & 1))
                            bst2<kNT>(s.soc, soc_a, sv[j - 1], sv[j], (uint32_t)(j - 1) * (uint32_t)E * 8u);
                        if (j == H) bst<kNT>(s.soc, soc_b, sv[j], (uint32_t)(NC - 2) * (uint32_t)E * 8u);
                    } else {
                        bst<kNT>(s.soc, (uint32_t)soc_index(c, el1, NC, E) * 8u, sv[j]);
                    }
                    o_row[k_soc + c] = (float)r.soc;
                    o_row[k_soc + NC + c] = departure_obs<PK>((PK && !occ) ? 0u : w[j]);
                    n_nonexist += r.nx;
                    fl |= r.fl;
                    if (L > 1) qv[L > 1 ? j : 0] = r.q;
                    // the lane's own penalties in charger order; kPairs: the last pair's come after the other
                    // lane's whole pairs (gather, below)
                    if (!kPairs || j < H) pen_v += r.q;
                    const bool ip = r.pw > 0.0;
                    seq_pos += r.pw;   // >= 0 here (the float32 product of a >= 0, or 0.0): adding it is exact
                    n_pos += ip ? 1 : 0;
                    pmin = __builtin_fmin(pmin, ip ? r.pw : __builtin_inf());
                    // chargers in order: charger j waits only for its own loads.  A/B of scheduling groups
                    // (profiles/r03_ab_wide_sched_groups.txt): config 5 22.6-22.7 us with one or two chargers
                    // per group, 22.8 with five, 27.1 with no barrier in a lane's 25 chargers; the headline
                    // within noise
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            // numpy sums fewer than 8 positive powers in order: one lane's running sum is that sum; two lanes'
            // partial sums combined are that sum only when one of them is empty or the sum is exact
            bool split = false;
            if constexpr (L > 1) {
                // the other lanes' totals (exact combinations), and their penalties after the first lane's own,
                // in charger order (adding a +0.0 term is exact)
                const double seq_own = seq_pos, pmin_own = pmin;
                const int n_own = n_pos;
                const uint32_t nx_own = n_nonexist, fl_own = fl;
                int with_pos = n_own > 0 ? 1 : 0;
                auto gather = [&](auto kc) {
                    constexpr int K = decltype(kc)::value;
                    const int nk = (int)from_part<L, K>((uint32_t)n_own);
                    with_pos += nk > 0 ? 1 : 0;
                    n_pos += nk;
                    seq_pos += from_part<L, K>(seq_own);
                    pmin = __builtin_fmin(pmin, from_part<L, K>(pmin_own));
                    n_nonexist += from_part<L, K>(nx_own);
                    fl |= from_part<L, K>(fl_own);
#pragma unroll
                    for (int j = 0; j < (kPairs ? H : CPL); ++j) {
                        const double qk = from_part<L, K>(qv[L > 1 ? j : 0]);
                        pen_v = leader ? pen_v + qk : pen_v;
                    }
                };
                gather(std::integral_constant<int, 1>{});
                if constexpr (L > 2) {
                    gather(std::integral_constant<int, 2>{});
                    gather(std::integral_constant<int, 3>{});
                }
                if constexpr (kPairs) {   // the last pair: charger N - 2 (this lane), then N - 1 (the other)
                    const double qk = from_part<L, 1>(qv[L > 1 ? H : 0]);
                    pen_v = leader ? (pen_v + qv[L > 1 ? H : 0]) + qk : pen_v;
                }
                split = with_pos > 1;
            }
            p_ch = seq_pos;
            const bool pos_slow = live && leader && (n_pos >= 8 || split) && !(seq_pos <= pmin * 0x1.0p28);
            if (__builtin_amdgcn_ballot_w64(pos_slow)) {   // wave-uniform: rare
                if (pos_slow) {
                    // the compacted positive powers again, in charger order: an occupied charger charging with
                    // a > 0 under bounded charging bills pc (charger.py:58-94); nothing else is positive here
                    PairwiseSum pos;
                    pos.init();
#pragma unroll 1
                    for (int c = 0; c < NC; ++c) {
                        const RecOff ro = rec_off(c, NC, E, el1);
                        const uint32_t wc = PK ? bld16(rec_t, ro.v, ro.s)
                                               : bld(s.word + plane, el4, (uint32_t)c * (uint32_t)E * 4u);
                        const float a = a_row[c];
                        const double pc = charging_power(p, a);
                        if ((wc & W_OCC) && p.bounded && a > 0.0f && pc > 0.0) pos.push(pc);
                    }
                    p_ch = pos.result();
                }
            }
        } else {
            // a wave with a discharging action: numpy's pairwise order for both signs (PairwiseSum), one
            // charger at a time on the env's first lane, its inputs re-read from memory and the actions tile
            PairwiseSum pos, neg;
            pos.init();
            neg.init();
            if (live && leader) {
#pragma unroll 1
                for (int c = 0; c < NC; ++c) {
                    const uint32_t r4 = (uint32_t)c * (uint32_t)E * 4u, r8 = 2u * r4;
                    const SocOff so = soc_off(c, NC, E, el8);
                    const RecOff ro = rec_off(c, NC, E, el1);
                    const uint32_t wc = PK ? bld16(rec_t, ro.v, ro.s) : bld(s.word + plane, el4, r4);
                    const double auxc = PK ? 0.0 : bld(s.aux + plane, el8, r8);
                    const double runc = bld(s.soc, so.v, so.s);
                    const double reqc = REQ ? bld(s.req + plane, el8, r8) : (p.req_zero ? 0.0 : 1.0);
                    const uint32_t capi = cap_field<PK>(wc);
                    const bool occ = (wc & W_OCC) != 0;
                    const ChargerResult r = charger_step<true, true, false, PK>(p, PK ? (wc & ~W_STATIC) : wc, auxc, runc,
                                                                                reqc, a_row[c], t, recip_cap((double)capi));
                    bst<kNT>(s.soc, so.v, (PK && !occ) ? (double)rec_soc(wc) : r.soc, so.s);
                    o_row[k_soc + c] = (float)r.soc;
                    o_row[k_soc + NC + c] = departure_obs<PK>((PK && !occ) ? 0u : wc);
                    n_nonexist += r.nx;
                    fl |= r.fl;
                    pen_v += r.q;
                    if (r.pw > 0.0) pos.push(r.pw);
                    if (r.pw < 0.0) neg.push(r.pw);
                }
            }
            p_ch = pos.result();
            p_dis = neg.result();
        }
        SNG_WSTAMP(2);
        if (live && leader) {
            pen_v += (t == 0) ? pen0_l : 0.0;   // python index -1 slot; every per-charger term is 0 at t = 0
            env_tail<false, true>(p, s, info, e0, (uint32_t)le, el1, el8, t, ratio, p.bess ? bess_l : 0.0, bess_action,
                                  p_ch, p_dis, pen_v, 100.0 * (double)n_nonexist, fl, o_row, k.v, fpv, fpr,
                                  info.episode_return ? ret_l : 0.0, 0.0, reward, done, &bs);
        }
        SNG_WSTAMP(3);
        wave_lds_fence();
        copy_out<kWave>(obs + e0 * O, s_obs, nw * O, vec_io != 0, lane);
        SNG_WSTAMP(4);
    }
};

// L lanes per env (1, 2 or 4): lane `part` of an env steps chargers [part * CPL, min(NC, (part + 1) * CPL)),
// CPL = ceil(NC / L).  The env's lanes are adjacent (one DPP quad); the partial charging sums, counts and
// minima combine exactly on the first lane (a sum the exactness test accepts is exact in any order, and
// fewer than 8 powers are numpy's in-order sum when one lane holds them all), the first lane adds the
// other lanes' vehicle penalties after its own in charger order (Python's sum, penaliser.py:55), and the
// rare exact-order paths run on the first lane over all chargers.  One group of 64 / L envs per wavefront;
// the register budget is sized for L waves per SIMD (every wave of the E = 65,536 grid resident at once).
// Measured and reverted (A/B on one box):
//   - two groups of 32 envs per wavefront at N = 10 (1,024 wavefronts, each group's loads issued before the
//     first group is stepped): 8.62-8.64 us per step in the graph against 6.68-6.71 us
//     (profiles/r04_ab_groups.txt);
//   - config 5 with four lanes per env and a 3-wave budget (166 VGPRs, no spills, 3 of the 4,096 waves per
//     SIMD resident): 29.6-29.8 us against 23.4 us with two lanes (profiles/r03_ab_config5_four_lanes.txt);
//   - round 5: two or four such wavefronts per workgroup (each with its own envs and LDS tiles, no barrier;
//     512 / 1,024 workgroups instead of 2,048): 6.79-6.80 / 6.99-7.03 us per step in the graph against
//     6.31-6.34 us with one (profiles/r05_ab_waves_per_workgroup.txt).
template <int NC, int L, bool PK, bool REQ, bool NOISE>
__global__ __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(L, L))) void
step_wide_kernel(const float *__restrict__ act, float *__restrict__ obs, double *__restrict__ reward,
                 uint8_t *__restrict__ done, int64_t E, int t, int vec_io, StepConst k, Params p, DeviceState s,
                 InfoPtrs info) {
    static_assert(L == 1 || L == 2 || L == 4, "one, two or four lanes per env");
    using Grp = WideGroup<NC, L, PK, REQ, NOISE>;
    using Lay = WideLds<NC, L>;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int lane = threadIdx.x;
    float *s_obs = lds + Lay::ACT;   // the actions tile, then the observation tile
    Grp g;
    const int64_t e0 = (int64_t)blockIdx.x * Grp::WENVS;   // the grid covers E: the wavefront has an env
    g.issue(e0, act, E, t, vec_io, p, s, info, lane);
    g.act_tile.commit(lds, lane);
    wave_lds_fence();
    g.run(lds, s_obs, obs, reward, done, E, t, vec_io, k, p, s, info, lane);
    SNG_WSTAMP_FLUSH(g.stamp_, 5);
    if (PK && t == 0 && p.bump_day && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_fetch_add(s.episode, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------
// The fused step: SmartNanogridEnv.step(actions) for BLOCK/L envs per workgroup.
// NC   = compile-time charger count (0: runtime p.n, L must be 1);
// L    = lanes per env;
// DIAG = also write the per-step diagnostics (SngInfo arrays).
// Every per-charger load of a lane's batch is issued before any of it is used, and the first
// batch before the action staging wait, so one lane keeps 3*CH + 2 requests in flight.
// ---------------------------------------------------------------------------------
// One wavefront per SIMD at the bench's population (1,024 waves), so the kernel may use the whole register
// file: amdgpu_waves_per_eu(1, 1) lets the wide stations' prefetched batch live in registers (at the
// default two waves per SIMD the compiler spilled it to scratch).
template <int NC, int L, bool DIAG, bool FAST, bool PK>
__global__ __launch_bounds__(step_block(NC)) __attribute__((amdgpu_waves_per_eu(1, 1))) void step_kernel(
    Params p, DeviceState s, InfoPtrs info,
                                                              const float *__restrict__ act, float *__restrict__ obs,
                                                              double *__restrict__ reward, uint8_t *__restrict__ done,
                                                              int64_t E, int t, int vec_io) {
    static_assert(L == 1 || NC > 0, "multi-lane envs need a compile-time charger count");
    using Lay = StepLds<NC, L>;
    constexpr int WENVS = Lay::WENVS;
    constexpr bool kRows = Lay::kRows;
    constexpr int CH = (L > 1) ? (NC + L - 1) / L : wide_batch(NC);
    // actions tile in one round: K float4 per lane covers WENVS * A floats for A <= NC + 1
    constexpr int KT = NC > 0 ? ((NC + 1) * WENVS + 4 * kWave - 1) / (4 * kWave) : 8;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = NC ? NC : p.n;
    const int A = p.act_dim, O = p.obs_dim;
    // the wavefront index is wave-uniform: readfirstlane keeps e0 and the row offsets scalar
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int le = lane / L, part = lane % L;
    const int64_t e0 = (int64_t)blockIdx.x * Lay::ENVS + (int64_t)wave * WENVS;   // this wave's first env
    if (e0 >= E) return;                                                           // wave-uniform
    const int nw = (int)((E - e0) < WENVS ? (E - e0) : WENVS);
    const int64_t e = e0 + le;
    const bool live = le < nw;
    const bool leader = part == 0;
    float *s_act = reinterpret_cast<float *>(reinterpret_cast<char *>(lds) + wave * Lay::wave_bytes(A, O));
    float *s_obs = reinterpret_cast<float *>(reinterpret_cast<char *>(s_act) + Lay::first_bytes(A));
    double *s_rcp = reinterpret_cast<double *>(s_obs + Lay::obs_floats(O));   // [256] 1/c (kRows)
    double *s_cst = s_rcp + (kRows ? 256 : 0);                    // [16] per-step constants (kRows)
    double *s_pos = s_cst + (kRows ? 16 : 0);                     // [WENVS][NC] compacted positive powers
    double *s_neg = s_pos + (kRows ? WENVS * NC : 0);             // [WENVS][NC] compacted negative powers
    double *s_pw = s_neg + (kRows ? WENVS * NC : 0);              // [WENVS][NC] per-charger powers (L > 1)
    double *s_q = reinterpret_cast<double *>(s_act);              // [WENVS][NC] penalty terms (L > 1)
    const uint32_t *__restrict__ word = s.word;
    const double *__restrict__ auxv = s.aux;
    const double *__restrict__ reqv = s.req;
    double *__restrict__ socv = s.soc;
    const size_t tbase = (size_t)t * n;
    const int cbeg = (L > 1) ? part * CH : 0;
    const int cend = (L > 1) ? ((cbeg + CH) < n ? (cbeg + CH) : n) : n;

    // Loads are issued oldest-needed-last: everything the LDS commits wait for (tables, actions
    // tile) is issued after the conditional loads and before the per-charger state, and no
    // branch separates it from the per-charger loads, so the wait before the commits is
    // vmcnt(#per-charger loads) and charger c's update starts as soon as its own loads land.
    // Non-live lanes load a valid env (E - 1) and discard it.
    const int64_t el = live ? e : E - 1;
    const uint32_t lo = (uint32_t)(el - e0);   // lane offset from the wave's first env
    const uint32_t el1 = (uint32_t)el, el4 = el1 * 4u, el8 = el1 * 8u;   // byte offsets of the env
    const uint32_t *__restrict__ word_t = word + tbase * (size_t)E;   // this step's timeline planes
    const double *__restrict__ aux_t = auxv + tbase * (size_t)E;
    // a packed day's records: plane t + 1 (sng_layout.h)
    const uint16_t *__restrict__ rec_t = packed_records(s) + (tbase + n) * (size_t)E;
    const double *__restrict__ req_t = reqv + tbase * (size_t)E;
    uint32_t w[CH];
    double aux[CH], run[CH], req[CH];
    auto load_state = [&](int c0) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
            const int c = c0 + j;
            if (c < cend) {
                const uint32_t r4 = (uint32_t)c * (uint32_t)E * 4u, r8 = 2u * r4;   // charger row
                if (PK) {   // packed device-day record (sng_layout.h)
                    const RecOff ro = rec_off(c, n, E, el1);
                    w[j] = bld16(rec_t, ro.v, ro.s);
                } else {
                    w[j] = bld(word_t, el4, r4);
                    aux[j] = bld(aux_t, el8, r8);
                }
                const SocOff so = soc_off(c, n, E, el8);   // the SoC state in charger pairs
                run[j] = bld(socv, so.v, so.s);
            } else {
                w[j] = 0u;
                aux[j] = run[j] = 0.0;
            }
        }
    };
    auto load_req = [&](int c0) {
        if (p.req_stream && !p.req_zero) {
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int c = c0 + j;
                req[j] = (c < cend) ? bld(req_t, el8, (uint32_t)c * (uint32_t)E * 8u) : 1.0;
            }
        } else {
            // no stream: 1.0 (requested SoC disabled, charging_station.py:230-232); a replayed day: the
            // cleared 0.0 (sng_layout.h, Params::req_zero)
            const double rq = p.req_zero ? 0.0 : 1.0;
#pragma unroll
            for (int j = 0; j < CH; ++j) req[j] = rq;
        }
    };
    auto load_batch = [&](int c0) {
        load_req(c0);
        load_state(c0);
    };
    // Wide single-lane stations (several batches): batch b + 1's loads are issued before batch b is
    // computed, so they land while it computes instead of after it (the loop is not unrolled: the
    // prefetched registers are copied into the batch's at the top of the next iteration).
    constexpr bool kPF = (L == 1) && !kRows && (NC > 0) && (CH < NC) && (NC % CH == 0);
    constexpr int PFN = kPF ? CH : 1;
    uint32_t wn[PFN];
    double auxn[PFN], runn[PFN], reqn[PFN];
    auto load_next = [&](int c0) {
        if constexpr (kPF) {
            const bool rq_live = p.req_stream && !p.req_zero;
            const double rq = p.req_zero ? 0.0 : 1.0;
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int c = c0 + j;
                const uint32_t r4 = (uint32_t)c * (uint32_t)E * 4u, r8 = 2u * r4;   // charger row
                if (PK) {
                    const RecOff ro = rec_off(c, n, E, el1);
                    wn[j] = bld16(rec_t, ro.v, ro.s);
                } else {
                    wn[j] = bld(word_t, el4, r4);
                    auxn[j] = bld(aux_t, el8, r8);
                }
                const SocOff so = soc_off(c, n, E, el8);
                runn[j] = bld(socv, so.v, so.s);
                reqn[j] = rq_live ? bld(req_t, el8, r8) : rq;
            }
        }
    };

    // 1. per-env values: pointer selects rather than branches (a disabled stream re-reads ratio)
    const double ratio = bld(s.ratio, el8);
    const double bess_l = bld(p.bess ? s.bess : s.ratio, el8);
    const double pen0_l = bld(t == 0 ? s.pen0 : s.ratio, el8);
    const double ret_l = bld(info.episode_return ? info.episode_return : s.ratio, el8);
    const double bess0 = DIAG ? bld((p.bess && t > 0 && info.bess_initial) ? s.bess0 : s.ratio, el8) : 0.0;
    const double bess = p.bess ? bess_l : 0.0;
    const double pen0 = (t == 0) ? pen0_l : 0.0;
    const double ret_prev = info.episode_return ? ret_l : 0.0;
    // 2. requested SoC of the first batch and the day's profile factors for t..t+3 (uniform
    //    branches, ahead of the tile)
    load_req(cbeg);
    double fpv[4] = {1.0, 1.0, 1.0, 1.0}, fpr[4] = {1.0, 1.0, 1.0, 1.0};
    if (p.noise) profile_factors(p, s, el8, t, fpv, fpr);
    // 3. tables and the wave's actions tile
    //    (wide stations: no 1/c table, the step constants in scalar registers -- see StepLds)
    constexpr int RCP_PER_LANE = kRows ? 256 / kWave : 0;
    double rcp_v[RCP_PER_LANE > 0 ? RCP_PER_LANE : 1];
#pragma unroll
    for (int k = 0; k < RCP_PER_LANE; ++k) rcp_v[k] = s.tables->recip[k * kWave + lane];
    const double cst_v = (kRows && lane < CST_COUNT) ? step_constant(s.tables, t, lane) : 0.0;
    double cst_r[CST_COUNT];
    if (!kRows) {
#pragma unroll
        for (int i = 0; i < CST_COUNT; ++i) cst_r[i] = step_constant(s.tables, t, i);   // uniform: s_load
    }
    TileStage<KT, kWave> act_tile;
    act_tile.issue(act + e0 * A, nw * A, vec_io != 0, lane);
    // 4. per-charger state of the first batch
    load_state(cbeg);
#pragma unroll
    for (int k = 0; k < RCP_PER_LANE; ++k) s_rcp[k * kWave + lane] = rcp_v[k];
    if (kRows && lane < CST_COUNT) s_cst[lane] = cst_v;
    const double *cst = kRows ? s_cst : cst_r;
    act_tile.commit(s_act, lane);
    wave_lds_fence();

    const float *a_row = s_act + le * A;
    float *o_row = s_obs + le * O;
    const float bess_action = p.bess ? a_row[n] : 0.0f;   // before the q rows reuse the tile
    const int k_soc = (p.pv ? 8 : 4);
    // the observation header needs only the PV ratio and this step's constants: written here,
    // while the chargers' loads are still in flight, instead of at the end of the env tail
    if (live && leader) write_obs_header(o_row, p, cst + CST_IRR, cst + CST_PN, ratio, fpv, fpr);
    PairwiseSum pos, neg;
    double seq_pos = 0.0, seq_neg = 0.0;
    int n_pos = 0, n_neg = 0;
    double *row_pos = s_pos + le * NC, *row_neg = s_neg + le * NC;
    if (!kRows) {
        pos.init();
        neg.init();
    }
    // one power into the pairwise-sum state (numpy order: compacted array of positives/negatives).
    // Rows: unconditional LDS stores at the current count (a slot is overwritten until its element
    // is kept) and select-based counters, so nothing here is addressed through a pointer select.
    auto add_power = [&](double pw) {
        if (kRows) {
            const bool ip = pw > 0.0, in = pw < 0.0;
            row_pos[n_pos] = pw;
            row_neg[n_neg] = pw;
            // + max(pw, 0) / + min(pw, 0): adds the kept element, or a zero that leaves the running
            // sum exactly unchanged (v_max/v_min return the non-NaN operand: a NaN power is
            // dropped, as numpy's P[P > 0] drops it)
            seq_pos += __builtin_fmax(pw, 0.0);
            seq_neg += __builtin_fmin(pw, 0.0);
            n_pos += ip ? 1 : 0;
            n_neg += in ? 1 : 0;
        } else {
            if (pw > 0.0) pos.push(pw);
            if (pw < 0.0) neg.push(pw);
        }
    };
    double pen_v = 0.0;
    uint32_t n_nonexist = 0;
    uint32_t fl = 0;
    if (live) {
        for (int c0 = cbeg; c0 < cend; c0 += CH) {
            if constexpr (kPF) {   // NC % CH == 0: every batch is full
                if (c0 != cbeg) {
#pragma unroll
                    for (int j = 0; j < CH; ++j) {
                        w[j] = wn[j];
                        if (!PK) aux[j] = auxn[j];
                        run[j] = runn[j];
                        req[j] = reqn[j];
                    }
                }
                if (c0 + CH < cend) load_next(c0 + CH);
            } else if (c0 != cbeg) {
                load_batch(c0);
            }
            // the batch's actions ahead of the LDS writes below (they issue back to back)
            float av[CH];
            double rc[CH];
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int c = c0 + j;
                av[j] = (c < cend) ? a_row[c] : 0.0f;
            }
            if (L > 1) wave_lds_fence();   // the q rows below reuse the actions tile
#pragma unroll
            for (int j = 0; j < CH; ++j) {
                const int c = c0 + j;
                if (c >= cend) break;
                // 1/cap from the LDS table here, not ahead with the actions: it needs charger j's
                // record, and reading every record's up front waited for all of them
                // (wide stations: recip_cap instead of the LDS table, exact all the same -- div_by_cap)
                rc[j] = kRows ? s_rcp[cap_field<PK>(w[j])] : recip_cap((double)cap_field<PK>(w[j]));
                // a packed day: the arrival SoC is the running SoC the step before stored (sng_layout.h)
                const bool occ = (w[j] & W_OCC) != 0;
                const uint32_t wj = PK ? (w[j] & ~W_STATIC) : w[j];
                const double aux_j = PK ? 0.0 : aux[j];
                const ChargerResult r = charger_step<FAST, true, false, PK>(p, wj, aux_j, run[j], req[j], av[j], t, rc[j]);
                const SocOff so = soc_off(c, n, E, el8);
                bst<kNT>(socv, so.v, (PK && !occ) ? (double)rec_soc(w[j]) : r.soc, so.s);
                if (DIAG) {   // 'Charger power values' and the SOC[c, t] the day record holds
                    if (info.charger_power) info.charger_power[(size_t)e * n + c] = r.pw;
                    if (info.vehicle_soc) info.vehicle_soc[(size_t)e * n + c] = r.soc;
                }
                o_row[k_soc + c] = (float)r.soc;
                o_row[k_soc + n + c] = departure_obs<PK>((PK && !occ) ? 0u : w[j]);
                n_nonexist += r.nx;
                fl |= r.fl;
                if (L == 1) {
                    pen_v += r.q;
                    add_power(r.pw);
                } else {
                    s_pw[le * NC + c] = r.pw;
                    s_q[le * NC + c] = r.q;
                }
                // chargers in order: charger j's arithmetic waits only for its own loads
                // (vmcnt counts down charger by charger) and overlaps the later chargers' loads;
                // left to interleave them, the scheduler hoisted work that waited for all loads
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
    if (L > 1) {
        // gather the env's lanes (same wavefront): counts and flag bits, then in-order
        // penalty / power sums by the leader from LDS
#pragma unroll
        for (int off = 1; off < L; off <<= 1) {
            n_nonexist += (uint32_t)__shfl_down((int)n_nonexist, off, L);
            fl |= (uint32_t)__shfl_down((int)fl, off, L);
        }
        wave_lds_fence();
        if (live && leader) {
            if (kRows) {
#pragma unroll
                for (int c = 0; c < NC; ++c) {
                    pen_v += s_q[le * NC + c];
                    add_power(s_pw[le * NC + c]);
                }
            } else {
                // wide stations: compact in place -- positives into the power row, negatives into
                // the penalty row; slot k <= c has been read before it is rewritten at step c
                double *pw_row = s_pw + le * NC, *q_row = s_q + le * NC;
#pragma unroll 10
                for (int c = 0; c < NC; ++c) {
                    const double qv = q_row[c], v = pw_row[c];
                    pen_v += qv;
                    pw_row[n_pos] = v;
                    q_row[n_neg] = v;
                    seq_pos += __builtin_fmax(v, 0.0);
                    seq_neg += __builtin_fmin(v, 0.0);
                    n_pos += (v > 0.0) ? 1 : 0;
                    n_neg += (v < 0.0) ? 1 : 0;
                }
            }
        }
    }
    if (live && leader) {
        // t = 0 reads the python index -1 slot (pen0); every per-charger term is 0 there, and
        // adding +0.0 / adding to +0.0 is exact, so this equals the reference's choice of sum
        pen_v += pen0;
        double p_ch, p_dis;
        if (kRows) {
            constexpr int W = (NC > 0 && NC <= 16) ? NC : 1;   // kRows: NC in [1, 16]
            p_ch = pairwise_row_c<W>(row_pos, n_pos, seq_pos);
            p_dis = pairwise_row_c<W>(row_neg, n_neg, seq_neg);
        } else if (L > 1) {
            p_ch = pairwise_row(s_pw + le * NC, n_pos, seq_pos);
            p_dis = pairwise_row(s_q + le * NC, n_neg, seq_neg);
        } else {
            p_ch = pos.result();
            p_dis = neg.result();
        }
        env_tail<DIAG>(p, s, info, e0, lo, el1, el8, t, ratio, bess, bess_action, p_ch, p_dis, pen_v,
                       100.0 * (double)n_nonexist, fl,
                       o_row, cst, fpv, fpr, ret_prev, bess0, reward, done);
    }
    wave_lds_fence();
    copy_out<kWave>(obs + e0 * O, s_obs, nw * O, vec_io != 0, lane);
    // a device-RNG day's first step advances the day counter its reset read (generate_kernel);
    // nothing in this launch reads it (done last: at the top it perturbed the prologue's schedule).
    // A replayed day (bump_day = 0) drew no counter value of its own.
    if (PK && t == 0 && p.bump_day && blockIdx.x == 0 && threadIdx.x == 0) *s.episode += 1;
}

// ---------------------------------------------------------------------------------
// Counter-based draws shared by the device generator and the t = 0 observation kernels: draw i
// of a stream is mix32(key + i * golden), three 32-bit multiplies (the earlier 64-bit SplitMix
// streams cost ~4x the VALU; the generator is bound by its dense timeline stores otherwise).
// ---------------------------------------------------------------------------------
struct HashStream {
    uint32_t key, ctr;
    __device__ __forceinline__ uint32_t next() { return mix32(key + (ctr++) * 0x9e3779b9u); }
};

__device__ __forceinline__ double u32_unit(uint32_t x) { return (double)x * 0x1.0p-32; }   // [0, 1)

__device__ __forceinline__ int below(uint32_t x, int n) {   // floor(x * n / 2^32)
    return (int)(((uint64_t)x * (uint64_t)n) >> 32);
}

constexpr uint32_t kDomainRatio = 0x7a710000u;    // a generated day's PV ratio
constexpr uint32_t kDomainReplay = 0x7a720000u;   // the PV ratio of a replayed day

// random.randint(0, 180) / 100 (smart_nanogrid_environment.py:349) of device day `day`
__device__ __forceinline__ double pv_ratio_draw(uint64_t seed, uint64_t ge, uint64_t day) {
    HashStream r2{stream_key(seed, ge, kDomainRatio, day), 0u};
    return (double)below(r2.next(), 181) / 100;
}

// The ratio a replayed device day redraws (reset(generate_new_initial_values=False) redraws
// random_pv_shift_ratio, smart_nanogrid_environment.py:347-349): replay number `replay` of the handle.
__device__ __forceinline__ double replay_ratio_draw(uint64_t seed, uint64_t ge, uint64_t replay) {
    HashStream r2{stream_key(seed, ge, kDomainReplay, replay), 0u};
    return (double)below(r2.next(), 181) / 100;
}

// ---------------------------------------------------------------------------------
// One env's Python `random` stream (RefStreams, tempered words, two blocks) on its lane: the day-end
// random.randint(0, 180) the last step owes (end_draw; smart_nanogrid_environment.py:181) and the
// reset's random.randint(0, 180) / 100 (draw; :349) -- _randbelow(181) as getrandbits(8) rejection.
// A block boundary without a ready successor is twisted on the lane (mt_twist_lane).  Returns the
// ratio (or `keep` when nothing is drawn) and stores the stream's new position.
// ---------------------------------------------------------------------------------
__device__ __noinline__ void mt_twist_lane(const uint32_t *A, uint32_t *B);
__device__ __forceinline__ double py_ratio_lane(const RefStreams &ps, int64_t e, bool end_draw, bool draw,
                                                double keep) {
    uint32_t *blk = ps.mt + (size_t)e * 2 * kMtN;
    const int32_t pos = ps.pos[e];
    int cur = (pos >> 16) & 1, mti = pos & kMtPosMask;
    bool ready = (pos & kMtNextReady) != 0;
    auto next = [&]() -> uint32_t {
        if (mti >= kMtN) {
            if (!ready) mt_twist_lane(blk + cur * kMtN, blk + (cur ^ 1) * kMtN);
            cur ^= 1;
            mti -= kMtN;
            ready = false;
        }
        return blk[cur * kMtN + mti++];   // tempered in HBM
    };
    auto randint180 = [&]() -> int {
        uint32_t r;
        do {
            r = next() >> 24;
        } while (r >= 181u);
        return (int)r;
    };
    if (end_draw) (void)randint180();
    const double ratio = draw ? (double)randint180() / 100 : keep;
    ps.pos[e] = (cur << 16) | (ready ? kMtNextReady : 0) | mti;
    return ratio;
}

// ---------------------------------------------------------------------------------
// Observation at t = 0 after a reset (SmartNanogridEnv.reset -> __get_observations,
// smart_nanogrid_environment.py:349-351): SOC[c, 0] as generated, departure times at 0.
// mode (Obs0Mode, sng_layout.h) says where the PV ratio comes from and who advances the day
// counter; replay = the handle's replay number (OBS0_REPLAY of a device day), else -1.
// ---------------------------------------------------------------------------------
template <int BLOCK, bool PK>
__global__ __launch_bounds__(BLOCK) void observe0_kernel(Params p, DeviceState s, float *__restrict__ obs,
                                                         double *__restrict__ ep_return, int64_t E, int vec_io,
                                                         int mode, int64_t replay, RefStreams ps, int py) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int n = p.n, O = p.obs_dim;
    const int tid = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * BLOCK;
    const int nblk = (int)((E - e0) < BLOCK ? (E - e0) : BLOCK);
    const int64_t e = e0 + tid;
    float *o_row = lds + tid * O;
    if (tid < nblk) {
        const uint64_t ge = (uint64_t)(e + p.env_offset);
        double ratio;
        if (py) {   // reference-RNG days: the Python stream's draws (py bit 0: the ratio, bit 1: the day-end draw)
            ratio = py_ratio_lane(ps, e, (py & 2) != 0, (py & 1) != 0, 0.0);
            if (py & 1)
                s.ratio[e] = ratio;
            else
                ratio = s.ratio[e];
        } else if (mode == OBS0_DEVICE) {   // the day's draw, as the fused generator's t = 0 blocks make it
            ratio = pv_ratio_draw(p.seed, ge, *s.episode);
            s.ratio[e] = ratio;
        } else if (mode == OBS0_REPLAY && replay >= 0) {
            ratio = replay_ratio_draw(p.seed, ge, (uint64_t)replay);
            s.ratio[e] = ratio;
        } else {
            ratio = s.ratio[e];
        }
        // a generated day's python index -1 slot holds zeros; a replayed day's Requested_SOC is 0
        if (mode != OBS0_HOST) s.pen0[e] = 0.0;   // OBS0_GENERATED included
        double fpv[4] = {1.0, 1.0, 1.0, 1.0}, fpr[4] = {1.0, 1.0, 1.0, 1.0};
        if (p.noise) profile_factors(p, s, (uint32_t)e * 8u, 0, fpv, fpr);
        write_obs_header(o_row, p, s.tables->irr_norm, s.tables->price_norm, ratio, fpv, fpr);
        const int k = p.pv ? 8 : 4;
        const uint32_t *__restrict__ word = s.word;
        const double *__restrict__ auxv = s.aux;
        double *__restrict__ socv = s.soc;
        // batches of 16 chargers: all loads of a batch issued before its stores (t = 0 slice); a packed
        // day's two planes are both loaded up front (the plane-0 record is used only where plane 1 is
        // occupied), so a batch is one memory round trip (config-5 reset 293 -> 257 us, A/B)
        constexpr int B = 16;
        for (int c0 = 0; c0 < n; c0 += B) {
            uint32_t w[B];
            double aux[B];
            if (PK) {   // packed device-day records (sng_layout.h): t = 0 is plane 1; plane 0 carries
                        // the SoC of the t = 0 arrivals
                const uint16_t *rec = packed_records(s);
                uint32_t r0[B], r1[B];
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    const int c = c0 + j < n ? c0 + j : n - 1;
                    const size_t ri = rec_index(c, e, n, E);   // charger quads (sng_layout.h)
                    r1[j] = rec[(size_t)n * E + ri];
                    r0[j] = rec[ri];
                }
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    w[j] = (r1[j] & W_OCC) ? r1[j] : 0u;   // an empty charger's record carries a SoC, not a departure
                    aux[j] = (r1[j] & W_OCC) ? (double)rec_soc(r0[j]) : 0.0;
                }
            } else {
#pragma unroll
                for (int j = 0; j < B; ++j) {
                    const int c = c0 + j < n ? c0 + j : n - 1;
                    w[j] = word[(size_t)c * E + e];
                    aux[j] = auxv[(size_t)c * E + e];
                }
            }
#pragma unroll
            for (int j = 0; j < B; ++j) {
                const int c = c0 + j;
                if (c < n) {
                    // the SoC state in charger pairs (sng_layout.h): one 16 B store per pair (c0 is even)
                    if (c + 1 < n && !(j & 1))
                        bst2<kNT>(socv, (uint32_t)soc_index(c, e, n, E) * 8u, aux[j], aux[j + 1 < B ? j + 1 : j]);
                    else if (c + 1 == n && !(j & 1))
                        bst<kNT>(socv, (uint32_t)soc_index(c, e, n, E) * 8u, aux[j]);
                    o_row[k + c] = (float)aux[j];
                    o_row[k + n + c] = departure_obs<PK>(w[j]);
                }
            }
        }
        if (p.bess) o_row[O - 1] = (float)s.bess[e];
        if (ep_return) ep_return[e] = 0.0;
    }
    // a host day: profile_kernel read the counter for this day's factors, so the next day draws the
    // next value (a device day's counter is advanced by its first step; a replay keeps its day's)
    if ((mode == OBS0_HOST || mode == OBS0_GENERATED) && blockIdx.x == 0 && tid == 0) *s.episode += 1;
    __syncthreads();
    copy_out<BLOCK>(obs + e0 * O, lds, nblk * O, vec_io != 0, tid);
}

// ---------------------------------------------------------------------------------
// Stochastic PV / price profiles of the day (build-defined, SngConfig.pv_noise / price_noise): the env's
// day keys prof_key[e] = {PV key, price key}, from which the step and observation kernels expand the factor
// of entry k (profile_factor_key).  Runs in every reset before observe0_kernel, which advances the day
// counter it reads.  Thread = env.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void profile_kernel(Params p, DeviceState s, int64_t E) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    const uint64_t day = *s.episode;
    const uint64_t env_seed = p.seed + (uint64_t)p.env_offset + (uint64_t)e;
    s.prof_key[2 * e] = stream_key(env_seed, 0, kDomainPV, day);
    s.prof_key[2 * e + 1] = stream_key(env_seed, 0, kDomainPrice, day);
}

// ---------------------------------------------------------------------------------
// Device RNG day generator: the reference's per-charger vehicle process
// (charging_station.py:200-279: arrival with p = 0.4 when the charger is free, arrival SoC
// U(0.1, 0.9), capacity U{15..119}, requested SoC, departure U{t+4/dt .. min(t+10/dt, T+1/dt)-1})
// with counter-based 32-bit hash streams (HashStream), one per (global env, charger, day).
// Thread = (env, charger); writes the dense packed-record (/ req) timeline.
// ---------------------------------------------------------------------------------
// An arrival happens iff round(rand() - 0.1) == 1, i.e. rand() > 0.6 (p = 0.4) at each free step.

constexpr int kGenBlock = 256;       // 4 waves of consecutive envs, same charger
// vehicles per charger and day: each stays >= 4/dt steps and leaves one empty step, so at most
// T / (4/dt + 1) + 1 <= 7 (checked on the host); slots for 8
constexpr int kDayVehicles = 8;
constexpr float kInvLog2Q = -1.3569154488567239f;   // 1 / log2(0.6)

// LDS slots per thread: the list's kDayVehicles entries and one more, which phase 2's look-ahead may
// read (never use) once the walk has reached the sentinel in slot 7
constexpr int kDaySlots = kDayVehicles + 1;
__host__ __device__ constexpr size_t generate_lds_bytes(bool with_req) {
    return (size_t)kDaySlots * kGenBlock * (sizeof(uint32_t) + sizeof(float) + (with_req ? sizeof(double) : 0));
}

// One vehicle's draws (charging_station.py:257-279), in stream order: the geometric wait from
// tfree to the arrival, arrival SoC, capacity + departure, requested SoC.  Phase 1 below and the
// t = 0 observation blocks share it, so both see the same first vehicle.
// Two 32-bit draws per vehicle (three with requested SoC), from a two-multiply hash (GenStream):
// the generator is bound by the VALU it issues (18.4 us for ~1,000 VALU per (env, charger) thread
// at 65,536 x 10), and the draws were a third of it.  x1's top 24 bits give the geometric wait, x2's
// top 24 bits the SoC (a float32 value in [0.1f, 0.9f], computed in float), and the 16 low bits of
// the two drive capacity (floor(r * 105 / 2^16)) and, through the low half of r * 105 (a bijection
// of r, as 105 is odd), the departure.
struct VehicleDraw {
    int ta, dep;
    uint32_t cap;
    double soc;          // code_soc(code)
    uint32_t req_draw;
    uint32_t code;       // the arrival SoC's 13-bit code (sng_layout.h)
};
__device__ __forceinline__ uint32_t mix32_gen(uint32_t x) {   // "lowbias32" (two multiplies, bijective)
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
struct GenStream {
    uint32_t key, ctr;
    __device__ __forceinline__ uint32_t next() { return mix32_gen(key + (ctr++) * 0x9e3779b9u); }
};
// Stream key of (seed, global env, charger, day) for the generator: one hash per (env, charger) over the
// index ge * 128 + c (unique for ge < 2^25 and c < 128, the ABI's maximum station), the day's seed hash k0
// offset by ge >> 25 beyond that.  k0 is wave-uniform (scalar).
__device__ __forceinline__ uint32_t gen_key(uint64_t seed, uint64_t ge, uint32_t c, uint64_t day) {
    const uint32_t k0 = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + (uint32_t)day * 0x9e3779b9u));
    return mix32((k0 + (uint32_t)(ge >> 25) * 0x85ebca6bu) ^ (((uint32_t)ge << 7) | c));
}
__device__ __forceinline__ VehicleDraw draw_vehicle(const Params &p, GenStream &rng, int tfree, int i4, int i10,
                                                    int i1) {
    VehicleDraw d;
    const uint32_t x1 = rng.next(), x2 = rng.next();
    const float u = ((float)(x1 >> 8) + 1.0f) * 0x1.0p-24f;   // (0, 1]
    d.ta = tfree + (int)(__log2f(u) * kInvLog2Q);               // floor: the product is >= 0
    // uniform(0.1, 0.9) on 8,192 float32 values (the packed record holds the code, sng_layout.h code_soc)
    d.code = x2 >> (32 - kSocCodeBits);
    d.soc = (double)code_soc(d.code);
    const uint32_t r = ((x1 & 0xffu) << 8) | (x2 & 0xffu);
    const uint32_t rc = r * 105u;
    d.cap = p.diff_caps ? 15u + (rc >> 16) : 40u;   // randint(15, 120)
    const uint32_t yd = (p.diff_caps ? rc : r) & 0xffffu;
    const int hi_c = d.ta + i10, hi_d = p.T + i1;
    const int high = hi_c < hi_d ? hi_c : hi_d;
    const int low = d.ta + i4;
    d.dep = (low >= high) ? low : low + (int)(__umul24(yd, (uint32_t)(high - low)) >> 16);   // 16 x 8 bits
    d.req_draw = p.req_enabled ? rng.next() : 0u;
    return d;
}

// The t = 0 observation of a device-RNG day, computed from the streams rather than read back from
// the timeline, so it runs as extra blocks of the generator's grid with no dependency on the
// timeline blocks (SmartNanogridEnv.reset -> __get_observations, smart_nanogrid_environment.py:
// 349-351): each charger's first vehicle, if it arrives at t = 0, gives SOC[c, 0] and the
// departure entry; the PV ratio, the day's profile factors, the header and the BESS entry; the
// running SoC is seeded and the day return zeroed.  64 envs per block, lane = env, and the block's
// four wavefronts split the row: wavefront 0 the header (PV ratio, profile factors, BESS entry),
// wavefronts 1-3 the chargers round-robin; profile entries go to all four.  Grid rows y = N .. N + 3
// cover a timeline block's 256 envs.  A thread's work is then a few vehicles, like a timeline
// thread's, instead of the whole station (one thread per env ran ~10x longer and finished last),
// no wavefront runs the header under a mask, and the 64-row tile (7.4 KB at N = 10) no longer caps
// the grid at 5 workgroups per CU.
constexpr int kObsParts = kGenBlock / kWave;       // wavefronts per observation block (threads per env)
constexpr int kObsEnvs = kGenBlock / kObsParts;    // envs per observation block
constexpr int kObsBlocks = kGenBlock / kObsEnvs;   // observation blocks per 256 envs
__device__ __forceinline__ void observe_day0(const Params &p, const DeviceState &s, uint64_t seed, int64_t E, int i4,
                                             int i10, int i1, uint64_t day, float *__restrict__ obs,
                                             double *__restrict__ ep_return, int vec_io, float *lds, int q) {
    const int n = p.n, O = p.obs_dim;
    const int tid = threadIdx.x, part = __builtin_amdgcn_readfirstlane(tid / kWave), le = tid % kWave;
    const int64_t e0 = (int64_t)blockIdx.x * kGenBlock + (int64_t)q * kObsEnvs;
    if (e0 >= E) return;   // the whole block (before any barrier)
    const int nblk = (int)((E - e0) < kObsEnvs ? (E - e0) : kObsEnvs);
    const int64_t e = e0 + le;
    float *o_row = lds + le * O;
    if (le < nblk) {
        const uint64_t ge = (uint64_t)(e + p.env_offset);
        const uint64_t env_seed = p.seed + (uint64_t)p.env_offset + (uint64_t)e;
        if (p.noise && part == 0) {   // the day's profile keys (profile_kernel's)
            s.prof_key[2 * e] = stream_key(env_seed, 0, kDomainPV, day);
            s.prof_key[2 * e + 1] = stream_key(env_seed, 0, kDomainPrice, day);
        }
        if (part == 0) {
            const double ratio = pv_ratio_draw(seed, ge, day);
            s.ratio[e] = ratio;
            s.pen0[e] = 0.0;
            double fpv[4] = {1.0, 1.0, 1.0, 1.0}, fpr[4] = {1.0, 1.0, 1.0, 1.0};
            if (p.noise) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (p.pv_noise != 0.0) fpv[k] = profile_factor(env_seed, kDomainPV, day, k, p.pv_noise);
                    if (p.price_noise != 0.0) fpr[k] = profile_factor(env_seed, kDomainPrice, day, k, p.price_noise);
                }
            }
            write_obs_header(o_row, p, s.tables->irr_norm, s.tables->price_norm, ratio, fpv, fpr);
            if (p.bess) o_row[O - 1] = (float)s.bess[e];
            if (ep_return) ep_return[e] = 0.0;
        }
        const int k = p.pv ? 8 : 4;
        const uint32_t el8 = (uint32_t)e * 8u;
        // wavefronts 1..3: charger pairs part - 1, part + 2, ... (the SoC state's 16 B slots, sng_layout.h)
        for (int c0 = 2 * (part - 1); part > 0 && c0 < n; c0 += 2 * (kObsParts - 1)) {
            double soc0[2] = {0.0, 0.0};
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int c = c0 + i;
                if (c >= n) break;
                GenStream rng{gen_key(seed, ge, (uint32_t)c, day), 0u};
                const VehicleDraw d = draw_vehicle(p, rng, 0, i4, i10, i1);
                const bool occ0 = d.ta == 0;   // t = 0 < T always, and dep >= 4/dt > 0
                soc0[i] = occ0 ? d.soc : 0.0;
                o_row[k + c] = (float)soc0[i];
                o_row[k + n + c] = departure_obs(pack_word(occ0, occ0, false, 0u, occ0 ? (uint32_t)d.dep : 0u));
            }
            const SocOff so = soc_off(c0, n, E, el8);
            if (c0 + 1 < n)
                bst2<kNT>(s.soc, so.v, soc0[0], soc0[1], so.s);
            else
                bst<kNT>(s.soc, so.v, soc0[0], so.s);
        }
    }
    __syncthreads();
    copy_out<kGenBlock>(obs + e0 * O, lds, nblk * O, vec_io != 0, tid);
}

// Two phases per (env, charger):
//  1. the day's vehicles: the waiting time to the next arrival is the number of failed
//     Bernoulli(0.4) trials before the first success (geometric, one draw via -log2(u)/-log2(0.6)),
//     then arrival SoC, capacity and departure -- a few draws per vehicle instead of one per free
//     step, without the per-step divergent arrival branch;
//  2. the dense timeline, step by step, from the vehicle list kept in LDS.
// Grid (E / 256, rows + 4): blocks y < gen_rows(N) the timeline of charger quad y / 4, the last 4 rows the
// t = 0 observation (observe_day0).  The day counter is read here and advanced by the day's first step
// (step_kernel, t = 0), so no block of this grid waits on another.
// The timeline records leave as streaming (nontemporal) stores: reset 24.5-24.7 -> 22.5-22.7 us per day
// at 65,536 x 10 (A/B, one box), the steps' code and state staying in L2.  Diagnostic builds
// (round 2's -DSNG_GX_* builds, in commits before 8be1f55) split the reset's time: without the t = 0 observation blocks 24.3-24.9 us
// (they run beside the timeline blocks), without phase 1's draws 20.7, without the record stores 16-16.8.
// Write-through record stores (sc1 | nt, sc0 | sc1 | nt) left the day and the reset unchanged (A/B,
// profiles/r03_ab_generator_store_policy.txt).
constexpr int kGenRecPol = kNT;
// Timeline rows of the generator's grid (see generate_kernel): four rows of 64 envs per full charger quad; a
// last partial quad of w = N mod 4 chargers has 256 / w envs per row (w = 1, 2: one or two rows), or 64 envs
// with one lane in four idle (w = 3: four rows).
__host__ __device__ constexpr int gen_part_lanes(int w) { return w == 3 ? 4 : w; }   // lanes per env
__host__ __device__ constexpr int gen_rows(int n) { return 4 * (n / 4) + (n % 4 == 0 ? 0 : 4 * gen_part_lanes(n % 4) / 4); }
constexpr int kVehArrShift = 24;                   // vehicle list entry: arrival step (bits 24-31)
constexpr uint32_t kVehRecMask = 0x3fff8u;         // capacity (3-9) and departure (10-17)
// Vehicle list entries (LDS) are kept in the packed record's own layout: capacity in bits 3-9, departure
// step in 10-17 and arrival step in 24-31, so an occupied step's record is (entry & 0x3fff8 | flags) -
// t << 10 (the departure field becomes the steps left: it is > t while the vehicle is present, so nothing
// borrows, and below 64, so bits 16-17 clear); the arrival SoC is kept as the carry bits an empty record
// holds (rec_carry), computed once per vehicle in phase 1.  TT: the day's step count as
// a compile-time constant (the walk unrolled: 24 for the 1 h day), 0 for a runtime p.T; REQ: the
// requested-SoC stream.
template <int TT, bool REQ>
__global__ __launch_bounds__(kGenBlock) void generate_kernel(Params p, DeviceState s, uint64_t seed, int64_t E,
                                                             int i4, int i10, int i1, float *__restrict__ obs,
                                                             double *__restrict__ ep_return, int vec_io) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    uint32_t *s_veh = reinterpret_cast<uint32_t *>(lds);                      // [V][BLOCK] arr | cap<<8 | dep<<16
    uint32_t *s_car = s_veh + kDaySlots * kGenBlock;                           // [V][BLOCK] arrival SoC carry bits
    double *s_req = reinterpret_cast<double *>(s_car + kDaySlots * kGenBlock);     // [V][BLOCK] (REQ only)
    const int tid = threadIdx.x;
    // grid rows: the timeline first, row u of charger quad u / 4 and 64 envs [256 x + 64 (u mod 4), +64), thread =
    // (env tid / 4, charger tid mod 4 of the quad), so a wavefront's record stores are 16 envs x the quad's
    // records, contiguous in the quad layout (sng_layout.h rec_index); then the t = 0 observation blocks
    // (gridDim.y - gen_rows(N) of them).  Dispatched last, they fill the CUs behind the timeline's VALU-bound
    // waves instead of delaying them: reset 16.0-16.3 -> 15.5-15.6 us (A/B three times on one box, same days,
    // profiles/r06_ab_generator_obs_order.txt; round 3's kernel had measured the opposite order 0.6 % better)
    const int u = (int)blockIdx.y;
    const uint64_t day = *s.episode;
    if (u >= gen_rows(p.n)) {
        observe_day0(p, s, seed, E, i4, i10, i1, day, obs, ep_return, vec_io, lds, u - gen_rows(p.n));
        return;
    }
    const int full = 4 * (p.n / 4);                              // timeline rows of the full quads
    const int q4 = u < full ? (u >> 2) * 4 : p.n & ~3;          // the quad's first charger
    const int qw = p.n - q4 < 4 ? p.n - q4 : 4;                 // its width (the last quad may be partial)
    const int lpe = u < full ? 4 : gen_part_lanes(qw);          // lanes per env: 256 / lpe envs per row
    const int sub = u < full ? (u & 3) : u - full;              // the row's env block within the 256
    const int c = q4 + tid % lpe;
    const int64_t e = (int64_t)blockIdx.x * kGenBlock + (int64_t)sub * (kGenBlock / lpe) + tid / lpe;
    if (e >= E || c >= p.n) return;
    const uint64_t ge = (uint64_t)(e + p.env_offset);   // global env id
    GenStream rng{gen_key(seed, ge, (uint32_t)c, day), 0u};
    const int T = TT > 0 ? TT : p.T;
    const int n = p.n;

    // phase 1 (charging_station.py:200-279)
    int tfree = 0, nv = 0;
    for (int v = 0; v < kDayVehicles - 1; ++v) {   // the last slot holds the sentinel
        if (tfree >= T) break;
        const VehicleDraw d = draw_vehicle(p, rng, tfree, i4, i10, i1);
        if (d.ta >= T) break;
        s_veh[v * kGenBlock + tid] = ((uint32_t)d.ta << kVehArrShift) | (d.cap << P_CAP_SHIFT) | ((uint32_t)d.dep << P_DEP_SHIFT);
        s_car[v * kGenBlock + tid] = rec_carry(false, d.code);
        if (REQ) {
            const double lo = d.soc <= 0.9 ? d.soc + 0.1 : 1.0;
            s_req[v * kGenBlock + tid] = lo + (1.0 - lo) * u32_unit(d.req_draw);
        }
        nv = v + 1;
        tfree = d.dep + 1;   // the departure step stays empty (charging_station.py:239-251)
    }

    // slot nv: a sentinel that never arrives or departs (arrival = departure = 255), so phase 2 walks
    // the list without a per-step bound check or branch (nv <= 7 < kDayVehicles, checked on the host)
    s_veh[nv * kGenBlock + tid] = (0xffu << kVehArrShift) | (0xffu << P_DEP_SHIFT);
    s_car[nv * kGenBlock + tid] = 0u;
    if (REQ) s_req[nv * kGenBlock + tid] = 1.0;

    // phase 2: the timeline.  An empty step's record carries the SoC of a vehicle arriving at the
    // next step (sng_layout.h), and plane 0 that of a vehicle arriving at t = 0.  cur = list[v] is the
    // vehicle of step t (until it has departed), nxt = list[v + 1] the one after it, read from LDS a
    // step before it can be needed; the record is assembled branch-free.
    uint32_t cur = s_veh[tid], nxt = s_veh[kGenBlock + tid];
    uint32_t car_cur = s_car[tid], car_nxt = s_car[kGenBlock + tid];
    double req_cur = REQ ? s_req[tid] : 1.0, req_nxt = REQ ? s_req[kGenBlock + tid] : 1.0;
    int nx = kGenBlock + tid;   // the slot of list[v + 1]
    bool prev_occ = false;
    bool pen = false;   // step t is in the penalty-check list observe(t-1) built
    // step t occupied / its vehicle arriving at t, carried from step to step: step t + 1 is occupied iff
    // its vehicle arrives then (arr1) or step t's vehicle stays past t + 1
    bool occ = (cur >> kVehArrShift) == 0u, stat = occ;
    // penalty-check list built by observe(t-1) (charging_station.py:42-63) as one unsigned range
    // test on the steps the vehicle at t-1 had left: on_departure {1}, sparse {1..3}, dense any;
    // no_penalty never (lo = 256 > any remainder)
    const uint32_t pen_lo = (p.penalty_mode == SNG_PENALTY_NONE) ? 256u : 1u;
    const uint32_t pen_span = (p.penalty_mode == SNG_PENALTY_SPARSE) ? 2u
                              : (p.penalty_mode == SNG_PENALTY_DENSE) ? 254u : 0u;
    // the record slot (quad layout: the quad row in soffset, env and charger in the lane offset) and the
    // requested-SoC slot ([N][E] planes: charger row and env in the lane offset)
    const uint32_t el2 = ((uint32_t)e * (uint32_t)qw + (uint32_t)(c - q4)) * 2u;
    const uint32_t r2 = (uint32_t)q4 * (uint32_t)E * 2u;
    const uint32_t el8 = ((uint32_t)c * (uint32_t)E + (uint32_t)e) * 8u;
    uint16_t *rec = reinterpret_cast<uint16_t *>(s.aux);
    const size_t nE = (size_t)n * (size_t)E;
    // raw buffer stores: the plane in the V#, the quad row in soffset, the slot in the lane offset
    bst16<kGenRecPol>(rec, el2, ((cur >> kVehArrShift) == 0u) ? car_cur : 0u, r2);
#pragma unroll
    for (int t = 0; t < T; ++t) {
        // the vehicle of step t + 1: past the current departure, the next one (the list ends in a
        // sentinel that never arrives or departs)
        const bool adv = (uint32_t)(t + 1) > ((cur >> P_DEP_SHIFT) & 0xffu);
        const uint32_t v1 = adv ? nxt : cur;
        const uint32_t car1 = adv ? car_nxt : car_cur;
        const double req1 = adv ? req_nxt : req_cur;
        nx += adv ? kGenBlock : 0;   // list[v + 1] for step t + 1 (slot 8 at most, kDaySlots)
        const uint32_t nxt1 = s_veh[nx];
        const uint32_t car_nxt1 = s_car[nx];
        const double req_nxt1 = REQ ? s_req[nx] : 1.0;

        const uint32_t flags = W_OCC | (stat ? W_STATIC : 0u) | (pen ? W_PEN : 0u);
        // capacity and departure in place, the departure becoming the steps left (dep > t while the vehicle
        // is present, and dep - t <= 10 / dt < 64 fits the record's 6 bits: nothing borrows or spills)
        const uint32_t w_occ = ((cur & kVehRecMask) | flags) - ((uint32_t)t << P_DEP_SHIFT);
        const bool arr1 = (v1 >> kVehArrShift) == (uint32_t)(t + 1);   // step t + 1's vehicle arrives then
        const uint32_t carry = arr1 ? car1 : 0u;
        const uint32_t w_emp = (pen ? W_PEN : 0u) | carry;
        bst16<kGenRecPol>(rec + (size_t)(t + 1) * nE, el2, occ ? w_occ : w_emp, r2);
        // requested SoC timeline (sng_layout.h): Requested_SOC[c, t-1] at t >= 1 -- the step reads
        // it where W_PEN is set -- and Requested_SOC[c, T-1] in the t = 0 slot (written below)
        if (REQ && t > 0) bst(s.req + (size_t)t * nE, el8, prev_occ ? req_cur : 0.0);
        prev_occ = occ;
        // step t + 1's penalty check: occupied at t with dep - t steps left in [pen_lo, pen_lo + pen_span]
        // (w_occ's departure field holds dep - t; an empty charger is never in the list)
        pen = occ && (w_occ >> P_DEP_SHIFT) - pen_lo <= pen_span;
        occ = (occ && (uint32_t)(t + 1) < ((cur >> P_DEP_SHIFT) & 0xffu)) || arr1;
        stat = arr1;
        cur = v1;
        car_cur = car1;
        req_cur = req1;
        nxt = nxt1;
        car_nxt = car_nxt1;
        req_nxt = req_nxt1;
    }
    if (REQ) bst(s.req, el8, prev_occ ? req_cur : 0.0);
}

// ---------------------------------------------------------------------------------
// Bandwidth probe (diagnostics, sng_bandwidth_probe): the measured ceiling the step kernel's roofline is
// quoted against.  One float4 per thread: thread i reads in[i] when i < nr and writes out[i] when
// i < nw (nontemporal, the step's store policy), so one dispatch moves 16 (nr + nw) bytes.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void probe_copy_kernel(const float4 *__restrict__ in, float4 *__restrict__ out,
                                                         int64_t nr, int64_t nw) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    typedef float v4f __attribute__((ext_vector_type(4)));
    v4f v = {0.f, 0.f, 0.f, 0.f};
    if (i < nr) v = reinterpret_cast<const v4f *>(in)[i];
    if (i < nw) __builtin_nontemporal_store(v, reinterpret_cast<v4f *>(out) + i);
}

hipError_t launch_probe_copy(const void *in, void *out, int64_t nr, int64_t nw, hipStream_t stream, hipEvent_t a,
                             hipEvent_t b) {
    const int64_t n = nr > nw ? nr : nw;
    const dim3 grid((unsigned)((n + 255) / 256)), block(256);
    if (a && b)
        hipExtLaunchKernelGGL(probe_copy_kernel, grid, block, 0, stream, a, b, 0u, (const float4 *)in, (float4 *)out,
                              nr, nw);
    else
        hipLaunchKernelGGL(probe_copy_kernel, grid, block, 0, stream, (const float4 *)in, (float4 *)out, nr, nw);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------
// launch wrappers (called from sng_api.cpp)
// ---------------------------------------------------------------------------------
// Optional start/stop events: hipExtLaunchKernel stamps them with the dispatch's own
// begin/end timestamps, i.e. the kernel's device time.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};

// Stations of 10 chargers without V2X (the headline configuration) step through the wide kernel with two
// lanes per env: A/B at 65,536 x 10 x 24 (round 3's tools/ab_headline.sh, in commits before 8be1f55; three runs each) 6.47-6.51 us per step
// in the day graph vs 6.67-6.71 for the lean kernel, day 0.1749-0.1761 vs 0.1796-0.1803 ms; one lane per
// env 6.75-6.79, four 8.15-8.23.  With V2X a discharging action is routine, and the lean kernel's LDS rows
// keep numpy's order cheaper than the wide kernel's rolled re-read.
// The lean step kernel's configurations: a compile-time station of N <= 16, one lane per env, no
// diagnostics, NumPy-2 promotion with a power-of-two dt, no stochastic profiles.
static bool lean_step(const Params &p, bool diag) {
    const bool nc = p.n == 1 || p.n == 2 || p.n == 4 || p.n == 8 || (p.n == 10 && p.v2x) ||
                    p.n == 16;
    return nc && !diag && !p.legacy && p.dt_pow2 && !p.noise && !(p.lanes == 2 || p.lanes == 4);
}

template <int NC>
static void launch_lean(const Params &p, const DeviceState &s, const InfoPtrs &info, const Tables &tab,
                        const float *act, float *obs, double *reward, uint8_t *done, int64_t E, int t, int vec_io,
                        hipStream_t stream, const LaunchEvents *ev) {
    StepConst k;
    for (int i = 0; i < CST_COUNT; ++i) k.v[i] = step_constant(&tab, t, i);
    const bool req = p.req_stream && !p.req_zero;
    auto kern = p.packed ? (req ? step_lean_kernel<NC, true, true> : step_lean_kernel<NC, true, false>)
                         : (req ? step_lean_kernel<NC, false, true> : step_lean_kernel<NC, false, false>);
    const dim3 grid((unsigned)((E + kLeanBlock - 1) / kLeanBlock)), block(kLeanBlock);
    const uint32_t lds = (uint32_t)LeanLds<NC>::BYTES;
    if (ev)
        hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ev->start, ev->stop, 0u, act, obs, reward, done, E, t,
                              vec_io, k, p, s, info);
    else
        hipLaunchKernelGGL(kern, grid, block, lds, stream, act, obs, reward, done, E, t, vec_io, k, p, s, info);
}

// The wide lean step kernel's configurations: N = 50 (BASELINE config 5's station), one lane per env, no
// diagnostics, NumPy-2 promotion with a power-of-two dt; stochastic profiles allowed.
static bool wide_step(const Params &p, bool diag) {
    return (p.n == 50 || (p.n == 10 && !p.noise && !p.v2x)) && !diag && !p.legacy && p.dt_pow2 &&
           !(p.lanes == 2 || p.lanes == 4);
}

// Lanes per env of the wide lean step kernel: two (2,048 wavefronts at 65,536 envs, two per SIMD).
// A/B at config 5 (round 3's tools/wide_ab.sh, in commits before 8be1f55; two runs each): 1 lane 25.85-25.91 us per step in the day graph,
// 2 lanes 22.54-22.62, 4 lanes 30.36-30.49 (128 VGPRs: 40 spilled to scratch).
__host__ __device__ constexpr int wide_lanes(int) { return 2; }

template <int NC>
static void launch_wide(const Params &p, const DeviceState &s, const InfoPtrs &info, const Tables &tab,
                        const float *act, float *obs, double *reward, uint8_t *done, int64_t E, int t, int vec_io,
                        hipStream_t stream, const LaunchEvents *ev) {
    constexpr int L = wide_lanes(NC);
    StepConst k;
    for (int i = 0; i < CST_COUNT; ++i) k.v[i] = step_constant(&tab, t, i);
    const bool req = p.req_stream && !p.req_zero;
    const int v = (p.packed ? 4 : 0) | (req ? 2 : 0) | (p.noise ? 1 : 0);
    void (*kerns[8])(const float *, float *, double *, uint8_t *, int64_t, int, int, StepConst, Params, DeviceState,
                     InfoPtrs) = {
        step_wide_kernel<NC, L, false, false, false>, step_wide_kernel<NC, L, false, false, true>,
        step_wide_kernel<NC, L, false, true, false>,  step_wide_kernel<NC, L, false, true, true>,
        step_wide_kernel<NC, L, true, false, false>,  step_wide_kernel<NC, L, true, false, true>,
        step_wide_kernel<NC, L, true, true, false>,   step_wide_kernel<NC, L, true, true, true>};
    auto kern = kerns[v];
    using Lay = WideLds<NC, L>;
    constexpr int ENVS = Lay::WENVS;   // envs per wavefront
    const dim3 grid((unsigned)((E + ENVS - 1) / ENVS)), block(kWave);
    const uint32_t lds = (uint32_t)((size_t)(Lay::ACT + Lay::OBS) * 4);
    if (ev)
        hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ev->start, ev->stop, 0u, act, obs, reward, done, E, t,
                              vec_io, k, p, s, info);
    else
        hipLaunchKernelGGL(kern, grid, block, lds, stream, act, obs, reward, done, E, t, vec_io, k, p, s, info);
}

static void launch_lean_n(const Params &p, const DeviceState &s, const InfoPtrs &info, const Tables &tab,
                          const float *act, float *obs, double *reward, uint8_t *done, int64_t E, int t, int vec_io,
                          hipStream_t stream, const LaunchEvents *ev) {
    switch (p.n) {
        case 1: launch_lean<1>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 2: launch_lean<2>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 4: launch_lean<4>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 8: launch_lean<8>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 10: launch_lean<10>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        default: launch_lean<16>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev); break;
    }
}

template <int NC, int L, bool DIAG>
static void launch_step_t(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                          double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                          const LaunchEvents *ev) {
    using Lay = StepLds<NC, L>;
    const dim3 grid((unsigned)((E + Lay::ENVS - 1) / Lay::ENVS)), block(Lay::BLOCK);
    const uint32_t lds = (uint32_t)Lay::bytes(p.act_dim, p.obs_dim);
    const bool fast = !p.legacy && p.dt_pow2;
    auto kern = p.packed ? (fast ? step_kernel<NC, L, DIAG, true, true> : step_kernel<NC, L, DIAG, false, true>)
                         : (fast ? step_kernel<NC, L, DIAG, true, false> : step_kernel<NC, L, DIAG, false, false>);
    if (ev)
        hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ev->start, ev->stop, 0u, p, s, info, act, obs, reward,
                              done, E, t, vec_io);
    else
        hipLaunchKernelGGL(kern, grid, block, lds, stream, p, s, info, act, obs, reward, done, E, t, vec_io);
}

template <int NC, bool DIAG>
static void launch_step_l(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                          double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                          const LaunchEvents *ev) {
    switch (p.lanes) {
        case 4: launch_step_t<NC, 4, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 2: launch_step_t<NC, 2, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        default: launch_step_t<NC, 1, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
    }
}

template <bool DIAG>
static void launch_step_n(const Params &p, const DeviceState &s, const InfoPtrs &info, const float *act, float *obs,
                          double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                          const LaunchEvents *ev) {
    switch (p.n) {
        case 1: launch_step_t<1, 1, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 2: launch_step_l<2, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 4: launch_step_l<4, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 8: launch_step_l<8, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 10: launch_step_l<10, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 16: launch_step_l<16, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        case 50: launch_step_l<50, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
        default: launch_step_t<0, 1, DIAG>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev); break;
    }
}

SNG_DIAG_SET_STAMPS   // diagnostic builds: sng_debug_set_stamps

int step_lanes_supported(int n, int lanes) {
    const bool multi = (n == 2 || n == 4 || n == 8 || n == 10 || n == 16 || n == 50);
    return (lanes == 1 || (multi && (lanes == 2 || lanes == 4))) ? 1 : 0;
}

// The step kernel writes the diagnostics (DIAG) when any SngInfo array other than the flags and the
// day return is given.
static bool info_diag(const InfoPtrs &info) {
    return info.grid_power || info.p_charge || info.p_discharge || info.bess_soc || info.pen_vehicle ||
           info.pen_battery || info.grid_cost || info.total_cost || info.solar || info.bess_power ||
           info.bess_calc_power || info.nonexistent || info.bess_initial || info.charger_power || info.vehicle_soc;
}

hipError_t launch_step(const Params &p, const DeviceState &s, const InfoPtrs &info, const Tables &tab,
                       const float *act, float *obs, double *reward, uint8_t *done, int64_t E, int t, int vec_io,
                       hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop) {
    LaunchEvents evs{ev_start, ev_stop};
    const LaunchEvents *ev = (ev_start && ev_stop) ? &evs : nullptr;
    if (lean_step(p, info_diag(info))) {
        launch_lean_n(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev);
        return hipGetLastError();
    }
    if (wide_step(p, info_diag(info))) {
        if (p.n == 10)
            launch_wide<10>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev);
        else
            launch_wide<50>(p, s, info, tab, act, obs, reward, done, E, t, vec_io, stream, ev);
        return hipGetLastError();
    }
    if (info_diag(info))
        launch_step_n<true>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev);
    else
        launch_step_n<false>(p, s, info, act, obs, reward, done, E, t, vec_io, stream, ev);
    return hipGetLastError();
}

// The name rocprofv3 reports for the step kernel launch_step would dispatch next (the template
// arguments launch_step_n / launch_step_l / launch_step_t select).
int step_kernel_name(const Params &p, const InfoPtrs &info, char *buf, int len) {
    if (lean_step(p, info_diag(info)))
        return snprintf(buf, (size_t)len, "void sng::step_lean_kernel<%d, %s, %s>", p.n, p.packed ? "true" : "false",
                        (p.req_stream && !p.req_zero) ? "true" : "false");
    if (wide_step(p, info_diag(info)))
        return snprintf(buf, (size_t)len, "void sng::step_wide_kernel<%d, %d, %s, %s, %s>", p.n, wide_lanes(p.n),
                        p.packed ? "true" : "false", (p.req_stream && !p.req_zero) ? "true" : "false",
                        p.noise ? "true" : "false");
    int nc = 0, lanes = 1;
    switch (p.n) {
        case 2: case 4: case 8: case 10: case 16: case 50:
            nc = p.n;
            lanes = (p.lanes == 2 || p.lanes == 4) ? p.lanes : 1;
            break;
        case 1: nc = 1; break;
        default: nc = 0; break;
    }
    const bool fast = !p.legacy && p.dt_pow2;
    return snprintf(buf, (size_t)len, "void sng::step_kernel<%d, %d, %s, %s, %s>", nc, lanes,
                    info_diag(info) ? "true" : "false", fast ? "true" : "false", p.packed ? "true" : "false");
}

hipError_t launch_observe0(const Params &p, const DeviceState &s, float *obs, double *ep_return, int64_t E,
                           int vec_io, hipStream_t stream, int mode, int64_t replay, const RefStreams *ps = nullptr,
                           int py = 0) {
    const RefStreams no_streams{nullptr, nullptr};
    const RefStreams &pss = (py && ps) ? *ps : no_streams;
    if (!ps) py = 0;
    if ((size_t)round4(256 * p.obs_dim) * 4 <= 64 * 1024) {
        const dim3 grid((unsigned)((E + 255) / 256)), block(256);
        auto kern = p.packed ? observe0_kernel<256, true> : observe0_kernel<256, false>;
        hipLaunchKernelGGL(kern, grid, block, (size_t)round4(256 * p.obs_dim) * 4, stream, p, s, obs, ep_return, E,
                           vec_io, mode, replay, pss, py);
    } else {
        const dim3 grid((unsigned)((E + kWave - 1) / kWave)), block(kWave);
        auto kern = p.packed ? observe0_kernel<kWave, true> : observe0_kernel<kWave, false>;
        hipLaunchKernelGGL(kern, grid, block, (size_t)round4(kWave * p.obs_dim) * 4, stream, p, s, obs, ep_return, E,
                           vec_io, mode, replay, pss, py);
    }
    return hipGetLastError();
}

hipError_t launch_profiles(const Params &p, const DeviceState &s, int64_t E, hipStream_t stream);

// A whole device-RNG reset.  The t = 0 observation runs as extra blocks of the generator's grid
// while its [256][obs_dim] LDS tile stays small next to the vehicle lists (N <= 16: at most 42 KB,
// a few generator workgroups per CU still fit); wider stations keep profile_kernel and
// observe0_kernel as separate launches behind the generator.
hipError_t launch_generate(const Params &p, const DeviceState &s, uint64_t seed, int64_t E, int i4, int i10, int i1,
                           float *obs, double *ep_return, int vec_io, hipStream_t stream, hipEvent_t ev_start,
                           hipEvent_t ev_stop) {
    const size_t veh = generate_lds_bytes(p.req_enabled != 0), tile = (size_t)round4(kObsEnvs * p.obs_dim) * 4;
    const bool fused = tile <= 32 * 1024;   // up to 60 chargers (config 5's 50: 27.9 KB)
    const dim3 grid((unsigned)((E + kGenBlock - 1) / kGenBlock), (unsigned)(gen_rows(p.n) + (fused ? kObsBlocks : 0))),
        block(kGenBlock);
    const size_t lds = (fused && tile > veh) ? tile : veh;
    const bool req = p.req_enabled != 0;
    auto kern = p.T == 24 ? (req ? generate_kernel<24, true> : generate_kernel<24, false>)
                : (p.T == 96 && !req) ? generate_kernel<96, false>   // config 5's 15-minute day
                : (req ? generate_kernel<0, true> : generate_kernel<0, false>);
    if (fused && ev_start && ev_stop) {   // the one-launch reset, timed by its own dispatch timestamps
        hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ev_start, ev_stop, 0u, p, s, seed, E, i4, i10, i1, obs,
                              ep_return, vec_io);
        return hipGetLastError();
    }
    if (ev_start) (void)hipEventRecord(ev_start, stream);
    hipLaunchKernelGGL(kern, grid, block, lds, stream, p, s, seed, E, i4, i10, i1, obs, ep_return, vec_io);
    hipError_t e = hipGetLastError();
    if (!fused) {
        if (e == hipSuccess) e = launch_profiles(p, s, E, stream);
        // the PV ratio and pen0 of the day, from the streams, as the fused t = 0 blocks do
        if (e == hipSuccess) e = launch_observe0(p, s, obs, ep_return, E, vec_io, stream, OBS0_DEVICE, -1);
    }
    if (e == hipSuccess && ev_stop) e = hipEventRecord(ev_stop, stream);
    return e;
}

// ---------------------------------------------------------------------------------
// Reference-RNG days on the GPU (SngRngMode SNG_RNG_REFERENCE): numpy's MT19937 stream of each env
// (np.random.seed(seed + global env), RandomState's state and draw semantics, sng_mt.h restates them
// for the host) drives ChargingStation.generate_initial_vehicle_presence_per_charger
// (charging_station.py:200-279) draw for draw, and the day is encoded into the word / f64 aux (/ req)
// timeline exactly as the host encoder does it (sng_api.cpp encode_day).  Three kernels:
//   mt_seed_kernel     init_genrand per env (once per seeding)
//   mt_prepare_kernel  per env, one wavefront: the state one twist ahead into the other block (the
//                      twist's three dependent ranges, 64 words at a time, in LDS)
//   ref_day2_kernel    per env, one lane: the day's draws (phase 1) and its timeline (phase 2)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) { return mt_temper_word(y); }
__device__ __forceinline__ uint32_t mt_untemper(uint32_t y) { return mt_untemper_word(y); }

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b) {   // twist term of words kk, kk + 1
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

// B = twist(A), both 624 words (MT19937's in-place twist, its ranges computed out of place):
// B[k] = A[k+M] ^ mix(A[k], A[k+1]) for k < N-M; B[k] = B[k+M-N] ^ mix(A[k], A[k+1]) up to N-2;
// B[N-1] = B[M-1] ^ mix(A[N-1], B[0]).
__device__ __forceinline__ void mt_twist_wave(const uint32_t *A, uint32_t *B, int lane) {
    constexpr int NM = kMtN - kMtM;   // 227
    for (int k = lane; k < NM; k += kWave) B[k] = A[k + kMtM] ^ mt_mix(A[k], A[k + 1]);
    wave_lds_fence();
    for (int k = NM + lane; k < 2 * NM; k += kWave) B[k] = B[k - NM] ^ mt_mix(A[k], A[k + 1]);
    wave_lds_fence();
    for (int k = 2 * NM + lane; k < kMtN - 1; k += kWave) B[k] = B[k - NM] ^ mt_mix(A[k], A[k + 1]);
    wave_lds_fence();
    if (lane == 0) B[kMtN - 1] = B[kMtM - 1] ^ mt_mix(A[kMtN - 1], B[0]);
    wave_lds_fence();
}

// the same by one thread, in place of the stream's exhausted other block (a day that draws past two
// blocks: not reachable by the generator's draw counts, kept for completeness)
// (both blocks tempered, as the streams keep them)
__device__ __noinline__ void mt_twist_lane(const uint32_t *A, uint32_t *B) {
    constexpr int NM = kMtN - kMtM;
    auto a = [&](int k) { return mt_untemper(A[k]); };
    auto b = [&](int k) { return mt_untemper(B[k]); };
    for (int k = 0; k < NM; ++k) B[k] = mt_temper(a(k + kMtM) ^ mt_mix(a(k), a(k + 1)));
    for (int k = NM; k < kMtN - 1; ++k) B[k] = mt_temper(b(k - NM) ^ mt_mix(a(k), a(k + 1)));
    B[kMtN - 1] = mt_temper(b(kMtM - 1) ^ mt_mix(a(kMtN - 1), b(0)));
}

// np.random.seed(s): init_genrand(s & 0xffffffff); mti = N, so the first draw twists
__global__ __launch_bounds__(256) void mt_seed_kernel(RefStreams rs, uint64_t seed0, int64_t E) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= E) return;
    uint32_t *b = rs.mt + (size_t)e * 2 * kMtN;
    uint32_t x = (uint32_t)(seed0 + (uint64_t)e);
    b[0] = mt_temper(x);
    for (int i = 1; i < kMtN; ++i) {
        x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)i;
        b[i] = mt_temper(x);
    }
    rs.pos[e] = kMtN;   // block 0, mti = N
}

// Before a day: an exhausted current block (mti = N) is replaced by its successor, and the block after the
// current one is put into the other slot, so the day has >= 624 draws without a twist of its own.  The
// position word is cur << 16 | kMtNextReady | mti; kMtNextReady says the other slot already holds the
// current block's successor (a day of ~300 draws leaves it untouched), so most days need no twist here.
__global__ __launch_bounds__(256) void mt_prepare_kernel(RefStreams rs, int64_t E) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4][2][kMtN];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave), lane = threadIdx.x % kWave;
    const int64_t e = (int64_t)blockIdx.x * 4 + wave;
    if (e >= E) return;   // wave-uniform
    const int32_t pos = rs.pos[e];
    int cur = (pos >> 16) & 1, mti = pos & kMtPosMask;
    const bool next_ready = (pos & kMtNextReady) != 0;
    if (next_ready && mti < kMtN) return;   // nothing to prepare
    uint32_t *blk = rs.mt + (size_t)e * 2 * kMtN;
    uint32_t *A = lds[wave][0], *B = lds[wave][1];
    if (mti >= kMtN && next_ready) {   // the successor is in place: it becomes the current block
        cur ^= 1;
        mti -= kMtN;
    }
    // 16 B per lane: a block is 156 groups of 4 words
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    auto load_block = [&](int slot, uint32_t *dst) {
        for (int g = lane; g < kMtN / 4; g += kWave) {
            u32x4 x = *reinterpret_cast<const u32x4 *>(blk + slot * kMtN + 4 * g);
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = mt_untemper(x[i]);
            *reinterpret_cast<u32x4 *>(dst + 4 * g) = x;
        }
    };
    auto store_block = [&](int slot, const uint32_t *src) {
        for (int g = lane; g < kMtN / 4; g += kWave) {
            u32x4 x = *reinterpret_cast<const u32x4 *>(src + 4 * g);
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = mt_temper(x[i]);
            *reinterpret_cast<u32x4 *>(blk + slot * kMtN + 4 * g) = x;
        }
    };
    load_block(cur, A);
    wave_lds_fence();
    if (mti >= kMtN) {
        mt_twist_wave(A, B, lane);
        uint32_t *x = A;
        A = B;
        B = x;
        cur ^= 1;
        mti -= kMtN;
        store_block(cur, A);
    }
    mt_twist_wave(A, B, lane);
    store_block(cur ^ 1, B);
    if (lane == 0) rs.pos[e] = (cur << 16) | kMtNextReady | mti;
}

// One env's numpy stream inside ref_day2_kernel: RandomState.random_sample / uniform / randint
// (legacy, masked rejection) over the tempered words of the prepared blocks (sng_mt.h, host twin).
//
// The words reach the lane through a ring of 64 words in LDS, topped up for the whole wavefront at
// once: the draws of a day are data-dependent (a free step draws two words, an arrival ~10), so the
// 64 lanes of a wavefront desynchronise, and a global load per draw made every draw of every lane
// wait out a memory round trip (0.53 ms per day at any population size).  A lane's draw is an LDS
// read; when any lane's ring holds <= kTopUp words, every lane holding <= kRefill words commits the
// next kRefill words into its ring.  Those words were loaded into registers one refill earlier (pf:
// 8 aligned 16 B loads), so a refill waits for loads issued a refill ago, not for a fresh round trip:
// the wavefront that draws issues no global stores (the timeline is the writer wavefront's, see
// ref_day2_kernel), so nothing else is counted in vmcnt ahead of those loads.  A draw that finds the
// ring empty (a rejection streak) refills its lane the same way.
// Stream word q counts from the start of the day's current block: block k = q / 624 sits in slot
// (cur0 + k) & 1, and a 4-word group never straddles two blocks (624 = 4 * 156).  Blocks 0 and 1 are
// prepared (mt_prepare_kernel); a day that draws into block 2 or beyond twists it on its lane into the
// slot of block k - 2, which the ring has consumed by then (it runs at most 96 words ahead: 64 in the
// ring, 32 in registers).
// LDS layout ring[slot][lane]: lanes reading any slots hit distinct banks.
constexpr int kRing = 64;     // words per lane in LDS
constexpr int kRefill = 32;   // words per refill (8 aligned 16 B groups)
constexpr int kTopUp = 24;    // after a top_up every lane holds more than this: the peeks reach head + 23
static_assert(kTopUp + kRefill <= kRing, "ring sizes");
// RandomState.random_sample from two tempered words (numpy's rk_double: 53 bits, a >> 5 and b >> 6)
__device__ __forceinline__ double rand53(uint32_t wa, uint32_t wb) {
    const int32_t a = (int32_t)(wa >> 5), b = (int32_t)(wb >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}
template <int ENVS>
struct MtRingT {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    uint32_t *blk;
    uint32_t *ring;   // this lane's ring: ring[slot * ENVS], slot < kRing
    int cur0;
    int head, tail;   // stream words (from the current block's start) drawn / committed into the ring
    int q0;           // the day's first word (mti at the start)
    int avail;        // stream blocks materialised: 0 .. avail - 1
    u32x4 pf[kRefill / 4];   // words [tail, tail + kRefill), loaded ahead of their refill
    __device__ __forceinline__ void materialise(int last) {   // blocks up to that of word `last`
        const int kmax = last / kMtN;
        while (avail <= kmax) {   // rare: a day of more than ~1,000 draws
            mt_twist_lane(blk + ((cur0 + avail - 1) & 1) * kMtN, blk + ((cur0 + avail) & 1) * kMtN);
            ++avail;
        }
    }
    // pf <- words [tail, tail + kRefill): they span at most two blocks (word tail + 4g is in block k0 up to
    // offset 624)
    __device__ __forceinline__ void prefetch() {
        materialise(tail + kRefill - 1);
        const int k0 = tail / kMtN, off0 = tail - k0 * kMtN;
        const uint32_t *b0 = blk + ((cur0 + k0) & 1) * kMtN, *b1 = blk + ((cur0 + k0 + 1) & 1) * kMtN;
#pragma unroll
        for (int g = 0; g < kRefill / 4; ++g) {
            const int off = off0 + 4 * g;
            pf[g] = *reinterpret_cast<const u32x4 *>(off < kMtN ? b0 + off : b1 + (off - kMtN));
        }
    }
    // the day's start: the ring is empty (tail = the first word's aligned group), its first words in flight
    __device__ __forceinline__ void start(int mti) {
        head = q0 = mti;
        tail = mti & ~3;
        avail = 2;
        prefetch();
    }
    // this lane: the prefetched words into the ring (which then holds <= kRing), the next ones in flight
    __device__ __forceinline__ void refill_lane() {
#pragma unroll
        for (int g = 0; g < kRefill / 4; ++g)
#pragma unroll
            for (int i = 0; i < 4; ++i) ring[((tail + 4 * g + i) & (kRing - 1)) * ENVS] = pf[g][i];   // tempered
        tail += kRefill;
        prefetch();
    }
    // wave-uniform test: lanes holding <= kRefill words refill, so every lane then holds > kTopUp
    __device__ __forceinline__ void top_up() {
        if (__builtin_amdgcn_ballot_w64(tail - head <= kTopUp))
            if (tail - head <= kRefill) refill_lane();
    }
    __device__ __forceinline__ uint32_t next() {
        if (head >= tail) refill_lane();   // the ring ran dry inside one step (a rejection streak)
        const uint32_t y = ring[(head & (kRing - 1)) * ENVS];
        ++head;
        return y;
    }
    // word head + k, without advancing: valid for k <= kTopUp after a top_up
    __device__ __forceinline__ uint32_t peek(int k) const { return ring[((head + k) & (kRing - 1)) * ENVS]; }
    __device__ __forceinline__ double random() {
        const uint32_t a = next();
        return rand53(a, next());
    }
    __device__ __forceinline__ double uniform(double lo, double hi) { return lo + (hi - lo) * random(); }
    __device__ __forceinline__ int randint(int low, int high) {   // exclusive high; one value: no draw
        if (high - 1 - low == 0) return low;
        uint32_t mask = (uint32_t)(high - 1 - low);
        mask |= mask >> 1;
        mask |= mask >> 2;
        mask |= mask >> 4;
        mask |= mask >> 8;
        mask |= mask >> 16;
        const uint32_t rng = (uint32_t)(high - 1 - low);
        uint32_t v;
        while ((v = (next() & mask)) > rng) {
        }
        return low + (int)v;
    }
    // the stream position after the day, as MtLane kept it: the block of the last word drawn and the
    // words drawn from it (624 = exhausted, twisted lazily at the next draw); kMtNextReady when the
    // other slot holds that block's successor
    __device__ __forceinline__ int32_t position() const {
        if (head == q0) return (cur0 << 16) | kMtNextReady | q0;
        const int k = (head - 1) / kMtN;
        return (((cur0 + k) & 1) << 16) | (k + 1 < avail ? kMtNextReady : 0) | (head - k * kMtN);
    }
};
// kRefGroups groups of ENVS envs per workgroup (lanes >= ENVS mirror them), each with a drawing wavefront
// (wavefront g) and a timeline wavefront (wavefront kRefGroups + g).  One group per workgroup: the
// dispatcher then puts two drawing wavefronts (and a timeline one) on ~96 of the 1,024 SIMDs, and their
// workgroups set the kernel's span (84 us against a median of 68 us).  Four groups (a workgroup of 8
// wavefronts fills one CU, wavefronts w and w + 4 on one SIMD) placed every drawing wavefront beside a
// timeline one, but the workgroup's barriers then couple four drawing wavefronts, and the span stayed at
// 85 us (A/B, profiles/r05_ab_refday_two_wavefronts.txt).
constexpr int kRefGroups = 1;
constexpr int kRefBlock = 2 * kRefGroups * kWave;

// The same day in two phases per charger, as generate_kernel draws a device day: (1) the charger's
// vehicles, visiting only the steps that draw (a free step draws the arrival test, an arrival the
// vehicle's values; an occupied step and a departure step draw nothing, charging_station.py:200-279),
// into a per-lane list in LDS; (2) the word / f64 aux (/ req) timeline from the list, branch-free, step
// by step.  Round 2's steps-major kernel executed the arrival path under a mask in nearly every (charger,
// step) iteration of a wavefront; here a wavefront iterates once per draw step of its busiest lane
// (about 5 of a charger's 24 steps draw).  The stream is consumed draw for draw.
// Round 5: the phases run on two wavefronts of one workgroup.  The drawing wavefront (0) writes charger
// c's list into LDS buffer c & 1 and meets the timeline wavefront (1) at one barrier per charger; the
// timeline wavefront then writes charger c's timeline from that buffer while the drawing wavefront draws
// charger c + 1 into the other one.  Round 4's single wavefront issued ~50 timeline stores per charger,
// and on gfx9 stores count in vmcnt ahead of any later load, so the next charger's first ring refill
// waited for all of them to complete (~0.8 us per charger) and the stores did not overlap the draws.
constexpr int kRefVeh = 8;   // vehicles per charger-day (T / (4/dt + 1) + 1 <= 7 for every dt dividing 24 h) + sentinel
// Phase 1 reads each draw step's words from the ring in two batches of LDS reads instead of one round
// trip per word: after a top_up every lane still drawing holds more than kTopUp words, so the 10 words
// an arrival may need first (arrival test, SoC, the discarded uniform, four capacity candidates) and the
// 6 it may need next (requested SoC, four departure candidates) are peeked without a bound check.  A
// masked rejection (numpy's legacy bounded randint) takes the first of four candidates that passes; all
// four rejected (p < 0.2 % for a capacity, < 0.4 % for a departure) continues word by word.
// A step without a vehicle draws only its arrival test, so phase 1 tests the next kScan steps together
// (integer compares, arrives()) and takes the first arrival with its vehicle in the same iteration: a
// wavefront iterates ~5 times per charger-day instead of once per drawing step of its busiest lane (~15).
// Round 5 (A/B, reference reset obs-ready at 65,536 envs): kScan 2 0.133 ms, 3 0.124, 4 0.119-0.121,
// 5 0.117-0.118, 6 0.117-0.119 (with a larger top-up).
constexpr int kScan = 5;
// the furthest peek of an iteration: the arrival tests up to 2 kScan - 1, then from an arrival at scan
// position kScan - 1 (skip 2 (kScan - 1)) the capacity path's 10 words and the departure's 6
static_assert(2 * (kScan - 1) + 10 + 5 <= kTopUp, "phase 1's peeks stay inside a topped-up ring");
// round(random.rand() - 0.1) == 1 (charging_station.py:214-215) on the 53-bit draw K = (a >> 5) << 26 |
// (b >> 6), random.rand() = K / 2^53 (rk_double): fl(K / 2^53 - 0.1) > 0.5 is monotone in K and holds
// from K = 0x13333333333334 on (checked against the double expression at every K within 3,000 of it and
// at 10^5 random K; tests/test_ref_arrival_threshold.py)
constexpr uint64_t kArrive53 = 0x13333333333334ull;
__device__ __forceinline__ bool arrives(uint32_t wa, uint32_t wb) {
    return ((((uint64_t)(wa >> 5)) << 26) | (uint64_t)(wb >> 6)) >= kArrive53;
}
// Vehicle-list buffers of ref_day2_kernel: charger c's list is in buffer c mod D.  The drawing wavefront's
// lanes do not wait for each other at the end of a charger: a lane that has drawn charger c's vehicles goes
// on to charger c + 1 while the wavefront's slowest lane still draws charger c (D = 3: one charger ahead;
// the timeline wavefront reads the buffer of charger c - 1 meanwhile).  A wavefront then iterates about as
// often as its busiest lane over the whole station (~41 times a day, simulated) instead of the sum over the
// chargers of each one's busiest lane (~51).  With the requested-SoC lists (REQ) two buffers fit the LDS
// of four workgroups per CU, and the lanes keep in step charger by charger.
__host__ __device__ constexpr int ref_day2_lists(bool req) { return req ? 2 : 3; }
// LDS of ref_day2_kernel: the rings, then the list buffers ([V][ENVS] each: entry, arrival SoC, and the
// requested SoC with REQ)
__host__ __device__ constexpr size_t ref_day2_list_bytes(bool req, int envs) {
    return (size_t)kRefVeh * envs * (4 + 8 + (req ? 8 : 0));
}
__host__ __device__ constexpr size_t ref_day2_group_bytes(bool req, int envs) {
    return (size_t)kRing * envs * 4 + (size_t)ref_day2_lists(req) * ref_day2_list_bytes(req, envs);
}
__host__ __device__ constexpr size_t ref_day2_lds_bytes(bool req, int envs) {
    return (size_t)kRefGroups * ref_day2_group_bytes(req, envs);
}
static_assert(ref_day2_lds_bytes(true, 64) <= 160 * 1024 && ref_day2_lds_bytes(false, 64) <= 160 * 1024,
              "a ref_day2_kernel workgroup fits one CU's LDS");
template <int TT, bool REQ, int ENVS>
__global__ __launch_bounds__(kRefBlock) __attribute__((amdgpu_waves_per_eu(2))) void ref_day2_kernel(Params p, DeviceState s, RefStreams rs, int64_t E,
                                                             int i4, int i10, int i1) {
    extern __shared__ __attribute__((aligned(16))) uint32_t rd_lds[];
    // At most two wavefronts per SIMD: a VGPR count above 512 / 3 (v175 reserved here; the kernel needs ~160).
    // With room for three, the dispatcher stacked two drawing wavefronts and a timeline one on ~96 of the
    // 1,024 SIMDs and left others with one, and those SIMDs' workgroups set the span: 86.9 -> 77.5 us,
    // reference reset 0.128 -> 0.119 ms obs-ready (A/B, profiles/r05_ab_refday_two_wavefronts.txt).  This assumes
    // gfx950's 512 VGPRs per SIMD lane with an allocation granule of 8 (176 > 512 / 3); tests/test_kernel_resources.py
    // reads the built code object's VGPR count and fails when the cap no longer holds
    // (profiles/r06_kernel_resources.txt: without this line the compiler allocates 158 VGPRs, three per SIMD).
    asm volatile("v_mov_b32 v175, 0" ::: "v175");
    const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x / kWave);
    const int wv = w / kRefGroups, g = w % kRefGroups;   // wv 0 draws, 1 writes group g's timeline
    const int wl = (int)threadIdx.x % kWave;
    const int lane = wl % ENVS;   // the env slot; lanes >= ENVS of either wavefront mirror it
    const int rec = (int)blockIdx.x * kRefGroups + g;   // the group's index (diagnostic stamps)
    const int64_t e0 = (int64_t)rec * ENVS;
    const bool live = e0 + lane < E && wl < ENVS;
    const int64_t e = e0 + lane < E ? e0 + lane : E - 1;   // past E: env E - 1's stream, nothing stored
    // the group's LDS: its ring [kRing][ENVS], then its list buffers
    uint32_t *glds = rd_lds + (size_t)g * ref_day2_group_bytes(REQ, ENVS) / 4;
    uint32_t *rings = glds;
    // list buffer b (charger c's is c mod D): entries ta | cap << W_CAP_SHIFT | dep << W_DEP_SHIFT, then arrival
    // SoC, then requested SoC (REQ)
    constexpr int D = ref_day2_lists(REQ);
    auto list_veh = [&](int b) {
        return reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(glds) + (size_t)kRing * ENVS * 4 +
                                            (size_t)b * ref_day2_list_bytes(REQ, ENVS));
    };
    auto list_soc = [&](int b) { return reinterpret_cast<double *>(list_veh(b) + kRefVeh * ENVS); };
    auto list_req = [&](int b) { return list_soc(b) + kRefVeh * ENVS; };
    const int T = TT > 0 ? TT : p.T, n = p.n;
    const uint32_t pen_lo = (p.penalty_mode == SNG_PENALTY_NONE) ? 256u : 1u;   // as generate_kernel
    const uint32_t pen_span = (p.penalty_mode == SNG_PENALTY_SPARSE) ? 2u
                              : (p.penalty_mode == SNG_PENALTY_DENSE) ? 254u : 0u;
    const uint32_t el8 = (uint32_t)e * 8u;
    const size_t nE = (size_t)n * (size_t)E;
    // diagnostic builds: stamps 0 / 1 the drawing wavefront's start and end, 2 its ticks in phase 1 (6, 7 its
    // XCC id and HW_ID); 3 the timeline wavefront's ticks in phase 2, 4 its end, 5 its HW_ID | XCC id << 32
    SNG_WSTAMP_DECL;
    SNG_WSTAMP(0);
    if (wv == 0) {
        [[maybe_unused]] const unsigned long long t1_ = SNG_WNOW();
        MtRingT<ENVS> rng;
        const int32_t pos = rs.pos[e];
        rng.blk = rs.mt + (size_t)e * 2 * kMtN;
        rng.ring = rings + lane;
        rng.cur0 = (pos >> 16) & 1;
        rng.start(pos & kMtPosMask);
        // phase 1: every lane draws its chargers' vehicles, one iteration per step that draws, charger after
        // charger; the wavefront meets the timeline wavefronts once all its lanes are past charger k (barrier
        // k + 1: the workgroup's, so the groups' drawing wavefronts meet there too), and a lane draws charger c
        // only while c <= k + D - 2 (its buffer is free)
        int c = 0, cb = 0, t = 0, nv = 0;   // the lane's charger, its buffer (c mod D), step, vehicles so far
        int kb = 0;                          // barriers passed (wave-uniform): k above
        uint32_t *s_veh = list_veh(0);
        double *s_soc = list_soc(0), *s_req = list_req(0);
        while (kb < n) {
            if (c < n && c <= kb + D - 2) {
                rng.top_up();   // ballots over the lanes drawing: each then holds > kTopUp words
                // the next kScan steps' arrival draws at once: the first that arrives, the free steps before
                // it consumed together
                uint32_t a[2 * kScan];
#pragma unroll
                for (int k = 0; k < 2 * kScan; ++k) a[k] = rng.peek(k);
                int j = kScan;
#pragma unroll
                for (int kk = kScan - 1; kk >= 0; --kk) j = arrives(a[2 * kk], a[2 * kk + 1]) ? kk : j;
                const int skip = min(j, T - t);
                rng.head += 2 * skip;
                t += skip;
                if (t < T && j < kScan) {   // an arrival at step t
                    uint32_t w[10];   // from the arrival draw: w[0], w[1] are it (not reread)
#pragma unroll
                    for (int k = 2; k < 10; ++k) w[k] = rng.peek(k);
                    const double soc = 0.1 + (0.9 - 0.1) * rand53(w[2], w[3]);      // uniform(0.1, 0.9), :257-259
                    const double lo = soc <= 0.9 ? soc + 0.1 : 1.0;
                    // w[4], w[5]: the discarded uniform (:219)
                    uint32_t cap = 40u;
                    bool seq = false;   // the draws continue word by word (a rejection streak)
                    if (p.diff_caps) {   // randint(15, 120) (:267-269): mask 127, accept <= 104
                        int k = 4;
                        uint32_t cv = 0u;
#pragma unroll
                        for (int kk = 3; kk >= 0; --kk) {   // the first candidate that passes, without an index
                            const uint32_t x = w[6 + kk] & 127u;
                            k = (x <= 104u) ? kk : k;
                            cv = (x <= 104u) ? x : cv;
                        }
                        if (k < 4) {
                            cap = 15u + cv;
                            rng.head += 7 + k;
                        } else {
                            rng.head += 10;
                            cap = (uint32_t)rng.randint(15, 120);
                            seq = true;
                        }
                    } else {
                        rng.head += 6;
                    }
                    double rq = 1.0;
                    const int high = min(t + i10, T + i1), low = t + i4;             // :271-279
                    int dep = low;
                    if (!seq) {
                        uint32_t v[6];
#pragma unroll
                        for (int k = 0; k < 6; ++k) v[k] = rng.peek(k);
                        constexpr int U = REQ ? 2 : 0;
                        if (REQ) rq = lo + (1.0 - lo) * rand53(v[0], v[1]);       // uniform(lo, 1), :261-265
                        int used = U;
                        if (low < high && high - 1 - low > 0) {   // randint(low, high); one value draws nothing
                            const uint32_t span = (uint32_t)(high - 1 - low);
                            uint32_t mask = span;
                            mask |= mask >> 1;
                            mask |= mask >> 2;
                            mask |= mask >> 4;
                            mask |= mask >> 8;
                            mask |= mask >> 16;
                            int k = 4;
                            uint32_t dv = 0u;
#pragma unroll
                            for (int kk = 3; kk >= 0; --kk) {
                                const uint32_t x = v[U + kk] & mask;
                                k = (x <= span) ? kk : k;
                                dv = (x <= span) ? x : dv;
                            }
                            if (k < 4) {
                                dep = low + (int)dv;
                                used += k + 1;
                            } else {
                                rng.head += U + 4;
                                used = 0;
                                uint32_t x;
                                while ((x = (rng.next() & mask)) > span) {
                                }
                                dep = low + (int)x;
                            }
                        }
                        rng.head += used;
                    } else {
                        rq = REQ ? rng.uniform(lo, 1.0) : 1.0;
                        dep = (low >= high) ? low : rng.randint(low, high);
                    }
                    const int vi = nv < kRefVeh - 1 ? nv : kRefVeh - 2;   // at most 7 (see kRefVeh)
                    s_veh[vi * ENVS + lane] = (uint32_t)t | (cap << W_CAP_SHIFT) | ((uint32_t)dep << W_DEP_SHIFT);
                    s_soc[vi * ENVS + lane] = soc;
                    if (REQ) s_req[vi * ENVS + lane] = rq;
                    nv = vi + 1;
                    t = dep + 1;   // occupied until dep - 1; the departure step is empty and draws nothing
                }
                if (t >= T) {   // the charger's list is complete: the sentinel, then the next charger
                    s_veh[nv * ENVS + lane] = 0xffu | (0xffu << W_DEP_SHIFT);   // never arrives
                    s_veh[(nv + 1 < kRefVeh ? nv + 1 : nv) * ENVS + lane] = 0xffu | (0xffu << W_DEP_SHIFT);
                    ++c;
                    cb = cb + 1 == D ? 0 : cb + 1;
                    t = 0;
                    nv = 0;
                    s_veh = list_veh(cb);
                    s_soc = list_soc(cb);
                    s_req = list_req(cb);
                }
            }
            // every lane past charger k: its list is complete, and the timeline wavefront may take it
            while (kb < n && __builtin_amdgcn_ballot_w64(c <= kb) == 0) {
                __syncthreads();   // barrier k + 1 (the timeline wavefront's of charger k)
                ++kb;
            }
        }
        SNG_WACC(2, t1_);
        if (live) rs.pos[e] = rng.position();
    } else {
        for (int c = 0; c < n; ++c) {
            __syncthreads();   // charger c's list is complete, in buffer c mod D
            [[maybe_unused]] const unsigned long long t2_ = SNG_WNOW();
            const uint32_t *s_veh = list_veh(c % D);
            const double *s_soc = list_soc(c % D), *s_req = list_req(c % D);
            // phase 2: the timeline (encode_day, sng_api.cpp): cur = the vehicle of step t until step t has
            // passed its departure step, nxt the one after it (read a step ahead); a stay of zero steps
            // (dep == arrival, possible when 4/dt < 1) still marks its arrival step STATIC, as the host
            // encoder's arrival list does
            int v = 0;
            uint32_t cur = s_veh[lane], nxt = s_veh[ENVS + lane];
            double soc_cur = s_soc[lane], soc_nxt = s_soc[ENVS + lane];
            double req_cur = REQ ? s_req[lane] : 1.0, req_nxt = REQ ? s_req[ENVS + lane] : 1.0;
            bool prev_occ = false;
            uint32_t prev_rem = 0u;
            double prev_req = 0.0;
#pragma unroll
            for (int tt = 0; tt < T; ++tt) {
                const uint32_t ta = cur & 0xffu, dep = cur >> W_DEP_SHIFT;
                const bool adv = (uint32_t)(tt + 1) > dep;   // step t + 1 belongs to the next vehicle
                const int vr = v + 2 < kRefVeh ? v + 2 : kRefVeh - 1;
                const uint32_t nn = s_veh[vr * ENVS + lane];   // list[v + 2], for when nxt becomes current
                const double soc_nn = s_soc[vr * ENVS + lane];
                const double req_nn = REQ ? s_req[vr * ENVS + lane] : 1.0;
                const bool occ = (uint32_t)tt >= ta && (uint32_t)tt < dep;
                const bool arrived = (uint32_t)tt == ta;
                const bool running = !arrived && prev_occ;
                const uint32_t rem = occ ? dep - (uint32_t)tt : 0u;
                const bool pen = prev_rem - pen_lo <= pen_span;   // prev_rem = 0: empty at t-1
                const size_t plane = (size_t)tt * nE;
                // every lane stores: a lane that is not live mirrors a live one (the same env's stream, so
                // the same values to the same addresses)
                {
                    // plain global stores (a uniform plane pointer + the env): one buffer descriptor per plane
                    // would not fit the SGPRs of the unrolled walk
                    const size_t row = plane + (size_t)c * (size_t)E;
                    s.word[row + (size_t)e] = pack_word(occ, !running, pen, occ ? (cur >> W_CAP_SHIFT) & 0xffu : 0u, rem);
                    s.aux[row + (size_t)e] = (occ && !running) ? soc_cur : 0.0;
                    if (REQ && tt > 0) s.req[row + (size_t)e] = prev_req;   // Requested_SOC[c, t-1]
                }
                prev_occ = occ;
                prev_rem = rem;
                prev_req = occ ? req_cur : 0.0;
                v += adv ? 1 : 0;
                cur = adv ? nxt : cur;
                soc_cur = adv ? soc_nxt : soc_cur;
                req_cur = adv ? req_nxt : req_cur;
                nxt = adv ? nn : nxt;
                soc_nxt = adv ? soc_nn : soc_nxt;
                req_nxt = adv ? req_nn : req_nxt;
            }
            if (REQ) bst(s.req, el8, prev_req, (uint32_t)c * (uint32_t)E * 8u);   // slot 0: Requested_SOC[c, T-1]
            SNG_WACC(3, t2_);
        }
    }
    const int t0 = w * kWave;   // the wavefront's first thread writes its stamps
    if (wv == 0) {
        SNG_WSTAMP(1);
        SNG_WSTAMP_PUT(0, stamp_[0], rec, t0);
        SNG_WSTAMP_PUT(1, stamp_[1], rec, t0);
        SNG_WSTAMP_PUT(2, stamp_[2], rec, t0);
        SNG_WSTAMP_PUT(6, (unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20), rec, t0);
        SNG_WSTAMP_PUT(7, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4), rec, t0);
    } else {
        SNG_WSTAMP(4);
        SNG_WSTAMP_PUT(3, stamp_[3], rec, t0);
        SNG_WSTAMP_PUT(4, stamp_[4], rec, t0);
        SNG_WSTAMP_PUT(5, (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                              ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32), rec, t0);
    }
}

// Envs per workgroup of ref_day2_kernel: each drawing wavefront's day is one serial chain (an env's stream
// is consumed charger after charger), so small populations spread over more, thinner workgroups.
static int ref_day2_envs(int64_t E) {
    return E >= 65536 ? 64 : E >= 16384 ? 32 : E >= 4096 ? 16 : 8;
}

// more than 64 KB of dynamic LDS (four groups of 64 envs: up to 144 KB) is allowed once per kernel; a
// refusal surfaces as the launch's error
template <int TT, bool REQ, int ENVS>
static void launch_ref_day2_envs(dim3 grid, dim3 block, size_t lds, hipStream_t stream, const Params &p,
                                 const DeviceState &s, const RefStreams &rs, int64_t E, int i4, int i10, int i1) {
    static const hipError_t set = hipFuncSetAttribute(reinterpret_cast<const void *>(ref_day2_kernel<TT, REQ, ENVS>),
                                                      hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      (int)ref_day2_lds_bytes(REQ, ENVS));
    (void)set;
    hipLaunchKernelGGL((ref_day2_kernel<TT, REQ, ENVS>), grid, block, lds, stream, p, s, rs, E, i4, i10, i1);
}

template <int TT, bool REQ>
static void launch_ref_day2(const Params &p, const DeviceState &s, const RefStreams &rs, int64_t E, int i4, int i10,
                            int i1, hipStream_t stream) {
    const int envs = ref_day2_envs(E);
    const int64_t per = (int64_t)envs * kRefGroups;   // envs per workgroup
    const dim3 grid((unsigned)((E + per - 1) / per)), block(kRefBlock);
    const size_t lds = ref_day2_lds_bytes(REQ, envs);
    switch (envs) {
        case 8: launch_ref_day2_envs<TT, REQ, 8>(grid, block, lds, stream, p, s, rs, E, i4, i10, i1); break;
        case 16: launch_ref_day2_envs<TT, REQ, 16>(grid, block, lds, stream, p, s, rs, E, i4, i10, i1); break;
        case 32: launch_ref_day2_envs<TT, REQ, 32>(grid, block, lds, stream, p, s, rs, E, i4, i10, i1); break;
        default: launch_ref_day2_envs<TT, REQ, 64>(grid, block, lds, stream, p, s, rs, E, i4, i10, i1); break;
    }
}

hipError_t launch_ref_seed(const RefStreams &rs, uint64_t seed0, int64_t E, hipStream_t stream) {
    hipLaunchKernelGGL(mt_seed_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, stream, rs, seed0, E);
    return hipGetLastError();
}

// One reference-RNG day of every env into the word / aux (/ req) planes; ratio, pen0 and the t = 0
// observation are the caller's (the Python stream stays on the host).
hipError_t launch_mt_prepare(const RefStreams &rs, int64_t E, hipStream_t stream) {
    hipLaunchKernelGGL(mt_prepare_kernel, dim3((unsigned)((E + 3) / 4)), dim3(256), 0, stream, rs, E);
    return hipGetLastError();
}

// prepare = false: the streams' blocks were prepared for this day already (sng_api.cpp prepares the next
// day's on a side stream while a day is stepped)
hipError_t launch_ref_day(const Params &p, const DeviceState &s, const RefStreams &rs, int64_t E, int i4, int i10,
                          int i1, bool prepare, hipStream_t stream) {
    if (prepare) {
        hipError_t e = launch_mt_prepare(rs, E, stream);
        if (e != hipSuccess) return e;
    }
    const bool req = p.req_stream != 0;
    if (p.T == 24) {
        if (req) launch_ref_day2<24, true>(p, s, rs, E, i4, i10, i1, stream);
        else launch_ref_day2<24, false>(p, s, rs, E, i4, i10, i1, stream);
    } else {
        if (req) launch_ref_day2<0, true>(p, s, rs, E, i4, i10, i1, stream);
        else launch_ref_day2<0, false>(p, s, rs, E, i4, i10, i1, stream);
    }
    return hipGetLastError();
}


__global__ void bump_day_kernel(DeviceState s) { *s.episode += 1; }

hipError_t launch_bump_day(const DeviceState &s, hipStream_t stream) {
    hipLaunchKernelGGL(bump_day_kernel, dim3(1), dim3(1), 0, stream, s);
    return hipGetLastError();
}

hipError_t launch_profiles(const Params &p, const DeviceState &s, int64_t E, hipStream_t stream) {
    if (!p.noise) return hipSuccess;
    const dim3 grid((unsigned)((E + 255) / 256)), block(256);
    hipLaunchKernelGGL(profile_kernel, grid, block, 0, stream, p, s, E);
    return hipGetLastError();
}

}  // namespace sng
