// sng_layout.h -- HBM layout shared by the host code and the HIP kernels.
//
// State of arrays, env index fastest everywhere so a wavefront's 64 lanes (64 envs)
// touch one contiguous 256 B / 512 B run per charger:
//
//   soc    f64 [N/2][E][2]  SOC[c, t] of the last stepped timestep (charger.py:16 array, one slot), in charger
//                           pairs: chargers 2k and 2k + 1 of env e are the 16 B at pair k's row, slot e, so a
//                           lane moves two of its env's chargers in one 16 B access (a wavefront: one 1 KiB run
//                           per instruction); with N odd the last charger is a row [E] of its own (soc_index)
//   bess   f64 [E]          BESS state of charge (persists across days)
//   bess0  f64 [E]          'Initial battery state of charge' of the current day
//   ratio  f64 [E]          random_pv_shift_ratio of the current day
//   pen0   f64 [E]          vehicle penalty at t=0 (reads the python index -1 slot; 0 for generated days)
//   word   u32 [T][N][E]    per charger-step scenario word (bits below)
//   aux    f64 [T][N][E]    per charger-step static SoC: the "previous" SoC when the word's
//                           STATIC bit is set (arrival: SOC[c, t] as generated), else the
//                           SOC[c, t] an unoccupied charger shows
//   rec    u16 [T+1][N/4][E][4]  device-RNG days only, in the aux buffer (`word` unused): one 2 B record
//                           per charger-step instead of 12 B in two planes (round 2: 4 B; round 4: 2 B),
//                           in charger quads: chargers 4k..4k+3 of env e are the 8 B at quad row k, slot
//                           e (a last partial quad of R = N mod 4 chargers: slots of 2R B; rec_index), so
//                           a lane reads four of its env's records in one 8 B load.
//                           Plane t + 1 is step t's record; plane 0 is a record "before the day".  An
//                           occupied charger's record holds OCC, STATIC, PEN, the capacity and the steps
//                           left (bits below).  An empty charger's record keeps OCC = 0 and PEN, and
//                           carries the arrival SoC of the vehicle that arrives at the next step as a
//                           13-bit code (0 when none): every arrival at t >= 1 follows an empty step (the
//                           departure step stays empty, charging_station.py:239-251), and plane 0 carries
//                           the t = 0 arrivals.  The step kernel stores the carried SoC as an empty
//                           charger's running SoC, so the arrival step reads it as the previous SoC; an
//                           empty charger shows 0 in the observation.  The device generator draws the
//                           arrival SoC as one of 8,192 float32 values spread evenly over [0.1, 0.9]
//                           (code_soc), so the code holds it exactly
//   req    f64 [T][N][E]    Requested_SOC[c, t-1] (read by the penalty check where W_PEN is set);
//                           the t = 0 slot, never read by a step, holds Requested_SOC[c, T-1] so the
//                           day can be exported (sng_get_scenario); only when enabled
//   flags  u32 [E]          sticky SNG_FLAG_* bits
//
// word bits (one u32 per charger and timestep):
//   bit 0      OCC     charger.occupancy[t] == 1
//   bit 1      STATIC  previous SoC comes from aux (t in vehicle_arrivals, or the slot before
//                      was not written this day) instead of the running SoC
//   bit 2      PEN     charger is in the penalty-check list that observe(t-1) built
//                      (charging_station.py:42-63); evaluated at step t
//   bits 8-15  CAP     vehicle capacity in kWh used at step t (integer, 15..119 or 40)
//   bits 16-23 DEP     departure time - t of the vehicle present at t (observation), 0 if none
//
// Packed record bits (u16, device-RNG days): bit 0 OCC, bit 1 STATIC, bit 2 PEN as in the word; occupied:
// bits 3-9 CAP (7 bits: 15..119 or 40), bits 10-15 the steps left to departure (dep - t <= 10 / dt <= 53
// for every dt of the 128-step timeline); empty: bits 3-15 the next step's arrival SoC code (code_soc).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SNG_HD __host__ __device__
#else
#define SNG_HD
#endif

namespace sng {

constexpr uint32_t W_OCC = 1u;
constexpr uint32_t W_STATIC = 2u;
constexpr uint32_t W_PEN = 4u;
constexpr int W_CAP_SHIFT = 8;
constexpr int W_DEP_SHIFT = 16;

constexpr int kMaxChargers = 128;   // numpy pairwise sum restated for n <= 128 (single level)
constexpr int kSlots = 25;          // charger.py:16-19
constexpr int kMaxT = 128;
constexpr int kPriceLen = 48;       // accountant.py:14, 49 (2T with the extended day)

SNG_HD inline uint32_t pack_word(bool occ, bool stat, bool pen, uint32_t cap, uint32_t dep) {
    return (occ ? W_OCC : 0u) | (stat ? W_STATIC : 0u) | (pen ? W_PEN : 0u) | ((cap & 0xffu) << W_CAP_SHIFT) |
           ((dep & 0xffu) << W_DEP_SHIFT);
}

// Element index of charger c, env e in the SoC state (charger pairs, above): pair row c & ~1 holds E
// 16 B slots, a last unpaired charger (N odd) a row of E 8 B slots.
SNG_HD inline size_t soc_index(int c, int64_t e, int n, int64_t E) {
    const int c0 = c & ~1;
    return (size_t)c0 * (size_t)E + (c0 + 2 <= n ? (size_t)e * 2u + (size_t)(c & 1) : (size_t)e);
}

// Element index of charger c, env e in a packed-record plane (charger quads, above).
SNG_HD inline size_t rec_index(int c, int64_t e, int n, int64_t E) {
    const int c0 = c & ~3;
    const int w = n - c0 < 4 ? n - c0 : 4;
    return (size_t)c0 * (size_t)E + (size_t)e * (size_t)w + (size_t)(c & 3);
}

constexpr int P_CAP_SHIFT = 3, P_DEP_SHIFT = 10;   // packed record fields (above)
constexpr uint32_t P_CAP_MASK = 0x7fu;
constexpr int P_SOC_SHIFT = 3, kSocCodeBits = 13;
// The arrival SoC of code k in [0, 8192): 0.1f + 0.8f * (k + 0.5) / 8192 in float32 (two roundings, no
// contraction: the library builds with -ffp-contract=off), a value in (0.1, 0.9).
SNG_HD inline float code_soc(uint32_t code) {
    const float u = ((float)code + 0.5f) * (1.0f / 8192.0f);   // exact: code + 0.5 and the scaling by 2^-13
    const float v = 0.8f * u;
    return 0.1f + v;
}
// An empty charger's packed record carrying arrival SoC code `code`.
SNG_HD inline uint32_t rec_carry(bool pen, uint32_t code) { return (pen ? W_PEN : 0u) | (code << P_SOC_SHIFT); }
// The arrival SoC an empty charger's record carries (meaningful when the next step is an arrival).
SNG_HD inline float rec_soc(uint32_t rec) { return code_soc((rec & 0xffffu) >> P_SOC_SHIFT); }
// A packed record's capacity and steps left as the word's fields (host decode).
SNG_HD inline uint32_t rec_cap(uint32_t rec) { return (rec >> P_CAP_SHIFT) & P_CAP_MASK; }
SNG_HD inline uint32_t rec_dep(uint32_t rec) { return (rec & 0xffffu) >> P_DEP_SHIFT; }

// Constant tables, in device memory, read with scalar (wave-uniform) loads.
struct Tables {
    double irr_norm[4 * kMaxT];    // irr[k] / irr_max          (pv_system_manager.py:81-85)
    double pv_power[4 * kMaxT];    // available_solar_power[k]  (:87-91)
    double price[4 * kMaxT];       // energy_price[0, k]        (accountant.py:38-40)
    double price_norm[4 * kMaxT];  // energy_price / max        (:42-46)
    double recip[256];             // 1.0 / c (correctly rounded), c = vehicle capacity; recip[0] = 0
    int32_t n_irr;
};

// Physical constants and switches, passed by value to every kernel.
struct Params {
    int32_t n;                // chargers
    int32_t T;                // steps per day
    int32_t obs_dim, act_dim;
    int32_t pv, bess, v2x, bounded, legacy, req_stream, penalty_mode;
    int32_t diff_caps, req_enabled;
    double dt;
    double rdt;               // 1 / dt, used only when dt is a power of two (x * rdt == x / dt exactly)
    int32_t dt_pow2;
    float dt_f;               // float32(dt) for the NEP 50 float32 product
    float ev_power_f, ev_eff_f;
    double ev_power, ev_eff;
    double bess_cap, bess_pmax_ch, bess_pmax_dis, bess_eff_ch, bess_eff_dis, bess_dod;
    double grid_w, bat_pen_w, sell_coef;
    int64_t env_offset;       // global index of env 0 of this handle (sharded runs)
    int32_t lanes;            // step kernel: lanes per environment (1, 2 or 4)
    int32_t noise;            // 1: stochastic PV / price profiles (DeviceState::prof_key is live)
    int32_t packed;           // 1: the day's timeline is packed records in `aux` (device-RNG days)
    int32_t req_zero;         // 1: Requested_SOC is 0 on every slot -- a replayed day: load_initial_values
                              //    (charging_station.py:119-136) does not restore what clear_initialisation_
                              //    variables (:138-150) zeroed, so no vehicle is ever insufficiently charged
    int32_t bump_day;         // 1: the loaded device-RNG day owns a day-counter value, which its first step
                              //    advances (0 for a replayed day: its counter value was advanced already)
    double pv_noise, price_noise;
    uint64_t seed;            // handle seed: env e's seed is seed + env_offset + e
};

// The reference RNG's numpy stream of every env on the device (SngRngMode SNG_RNG_REFERENCE): the
// MT19937 state of np.random.seed(seed + global env) as numpy's RandomState keeps it, in two blocks per
// env, env-major ([E][2][624] u32: one env's words are contiguous, so a lane drawing from its own
// stream reads consecutive words).  pos[e] = cur << 16 | mti: block `cur` holds the state whose
// tempered words mti..623 are the stream's next draws; mt_prepare_kernel puts the state one twist
// later into the other block before a day is drawn.  Python's `random` stream of every env (two or
// three draws a day) is kept the same way (py_ratio_kernel draws it).
// The blocks hold the state words TEMPERED (the stream's output words): the drawing kernels read their
// words as they are, and the twisting kernels untemper what they read and temper what they write
// (mt_temper_word / mt_untemper_word, a bijection).  Checkpoints export numpy's raw state.
struct RefStreams {
    uint32_t *mt;
    int32_t *pos;
};
constexpr int kMtN = 624, kMtM = 397;
SNG_HD inline uint32_t mt_temper_word(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}
SNG_HD inline uint32_t mt_untemper_word(uint32_t y) {
    y ^= y >> 18;                   // shifts of >= 16 bits undo in one step
    y ^= (y << 15) & 0xefc60000u;
    uint32_t t = y;                 // << 7: 5 steps cover 32 bits
#pragma unroll
    for (int i = 0; i < 4; ++i) t = y ^ ((t << 7) & 0x9d2c5680u);
    y = t;
    t = y ^ (y >> 11);              // >> 11: 3 steps
    return y ^ (t >> 11);
}
// RefStreams::pos word: cur << 16 | kMtNextReady | mti (mti <= 624)
constexpr int32_t kMtNextReady = 0x4000, kMtPosMask = 0x3fff;

struct DeviceState {
    double *soc, *bess, *bess0, *ratio, *pen0;
    uint32_t *word;
    double *aux, *req;
    uint32_t *flags;
    // the current day's profile keys [E][2] (PV, price: stream_key of the env's seed and the day), only when
    // Params::noise; the kernels expand factor k as profile_factor_key(key, k, sigma)
    uint32_t *prof_key;
    uint64_t *episode;        // device-side day counter for the device generator
    const Tables *tables;
};

// What observe0_kernel (the t = 0 observation of a day the fused generator did not write) does with
// the PV ratio, the t = 0 penalty and the day counter.
enum Obs0Mode : int32_t {
    OBS0_HOST = 0,     // host-RNG or injected day: ratio and pen0 were uploaded; advances the day counter
                       // (profile_kernel read it for this day's profile factors)
    OBS0_DEVICE = 1,   // device-RNG day of a wide station (generator launched without its t = 0 blocks):
                       // ratio drawn from the day's stream, pen0 = 0; the day's first step advances the counter
    OBS0_GENERATED = 3,   // reference-RNG day generated on the device: ratio uploaded, pen0 = 0 (a generated
                          // day's python index -1 slot holds zeros); advances the day counter like OBS0_HOST
    OBS0_REPLAY = 2,   // replayed day, reset(generate_new_initial_values=False): pen0 = 0, counter untouched;
                       // ratio uploaded (reference RNG) or drawn from the replay stream (device RNG)
};

struct InfoPtrs {
    double *grid_power, *p_charge, *p_discharge, *bess_soc, *pen_vehicle, *pen_battery, *grid_cost, *total_cost,
        *solar, *bess_power, *bess_calc_power, *nonexistent, *bess_initial;
    uint32_t *flags;
    double *episode_return;
    double *charger_power, *vehicle_soc;   // [E][N], DIAG only
    uint32_t *flag_any;                    // SngInfo.flag_summary [SNG_FLAG_SUMMARY_WORDS]: OR of the raised flags
};

}  // namespace sng
