/*
 * sng_oracle.c -- CPU restatement of the reference SmartNanogridEnv hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.  The product
 * (smart-nanogrid-gym_amd/) never links, loads or calls anything in oracle/.
 *
 * Parity pinning: checked against the golden vectors produced by running the
 * reference itself (tests/golden/make_golden.py -> tests/golden/<case>.npz, 21 cases)
 * and against the reference's recorded PPO episodes (tests/golden/kat/<file>.json).
 * The RNG restatement is checked draw-for-draw against numpy.random.RandomState
 * and Python's random.Random (tests/test_oracle_rng.py).
 *
 * It is a scalar, per-environment restatement that keeps the reference's own data
 * structures (25-slot per-charger arrays, ragged arrival/departure lists, the
 * penalty-check list computed during observe()) rather than the GPU's packed
 * layout, so that a layout bug in the product cannot be mirrored here.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * smart_nanogrid_gym/).  Compile with -O2 -ffp-contract=off (no FMA contraction).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORC_MAXV 32       /* max vehicles per charger per day (list capacity) */
#define ORC_MAXT 128
#define MT_N 624
#define MT_M 397

/* ------------------------------------------------------------------------------
 * MT19937: the generator behind numpy's legacy RandomState (np.random.*) and
 * Python's `random` module.  Standard Matsumoto-Nishimura recurrence.
 * ---------------------------------------------------------------------------- */
typedef struct { uint32_t mt[MT_N]; int mti; } orc_mt;

static void mt_init_genrand(orc_mt *s, uint32_t seed) {
    s->mt[0] = seed;
    for (int i = 1; i < MT_N; i++)
        s->mt[i] = 1812433253u * (s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) + (uint32_t)i;
    s->mti = MT_N;
}

static void mt_init_by_array(orc_mt *s, const uint32_t *key, int len) {
    mt_init_genrand(s, 19650218u);
    int i = 1, j = 0;
    for (int k = (MT_N > len ? MT_N : len); k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
        if (j >= len) j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        s->mt[i] = (s->mt[i] ^ ((s->mt[i - 1] ^ (s->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { s->mt[0] = s->mt[MT_N - 1]; i = 1; }
    }
    s->mt[0] = 0x80000000u;
    s->mti = MT_N;
}

static uint32_t mt_next(orc_mt *s) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    if (s->mti >= MT_N) {
        int kk;
        uint32_t y;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (s->mt[kk] & 0x80000000u) | (s->mt[kk + 1] & 0x7fffffffu);
            s->mt[kk] = s->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (s->mt[MT_N - 1] & 0x80000000u) | (s->mt[0] & 0x7fffffffu);
        s->mt[MT_N - 1] = s->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        s->mti = 0;
    }
    uint32_t y = s->mt[s->mti++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

/* np.random.seed(int): legacy seeding = init_genrand(seed & 0xffffffff). */
void orc_np_seed(orc_mt *s, uint32_t seed) { mt_init_genrand(s, seed); }

/* random.seed(int): init_by_array over the 32-bit words of |seed| (at least one). */
void orc_py_seed(orc_mt *s, uint64_t seed) {
    uint32_t key[2];
    int len = 0;
    do { key[len++] = (uint32_t)(seed & 0xffffffffu); seed >>= 32; } while (seed && len < 2);
    mt_init_by_array(s, key, len);
}

/* numpy random_sample()/rand(): 53-bit double from two draws. */
double orc_np_random(orc_mt *s) {
    int32_t a = (int32_t)(mt_next(s) >> 5), b = (int32_t)(mt_next(s) >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

/* numpy legacy uniform(low, high) = low + (high - low) * random_sample(). */
double orc_np_uniform(orc_mt *s, double low, double high) {
    double range = high - low;
    return low + range * orc_np_random(s);
}

/* numpy legacy randint(low, high) (exclusive high, int64): masked rejection on
 * 32-bit draws; no draw at all when the range is a single value. */
int64_t orc_np_randint(orc_mt *s, int64_t low, int64_t high) {
    uint64_t rng = (uint64_t)(high - 1 - low);
    if (rng == 0) return low;
    uint64_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4;
    mask |= mask >> 8; mask |= mask >> 16; mask |= mask >> 32;
    uint32_t v;
    while ((v = (mt_next(s) & (uint32_t)mask)) > (uint32_t)rng) {}
    return low + (int64_t)v;
}

/* Python random.randint(a, b) = a + _randbelow(b - a + 1) via getrandbits(k). */
int64_t orc_py_randint(orc_mt *s, int64_t a, int64_t b) {
    uint64_t n = (uint64_t)(b - a + 1);
    int k = 0;
    while ((n >> k) != 0) k++;          /* n.bit_length() */
    uint32_t r;
    do { r = mt_next(s) >> (32 - k); } while (r >= n);
    return a + (int64_t)r;
}

/* ------------------------------------------------------------------------------
 * Build-defined generalisation, off by default:
 *
 *   extended_day   days longer than 24 steps (dt < 1 h).  The reference cannot run them
 *                  (25-slot arrays, charger.py:16-19; 48-entry price table, accountant.py:49).
 *                  Here the per-charger arrays get T+1 slots (python index -1 -> slot T), the
 *                  price table gets 2T entries from the per-step tariff loop the reference
 *                  computes but does not use (accountant.py:61-68; models 1-4: the hourly
 *                  value of hour floor(i*dt)), the PV table is the dt-window mean as for any
 *                  dt (pv_system_manager.py:34-44), the generator is the reference's own
 *                  dt-scaled one, and the departure observation keeps its literal /24.
 *   pv_noise,      stochastic PV and price profiles: per env and day, every table entry k used
 *   price_noise    (reward at t, observation t..t+3) is scaled by f = 1 + sigma * z(k), z in
 *                  [-1, 1) from a counter-based hash of (env seed, day, domain, k).  sigma = 0
 *                  gives f = 1 exactly.
 *
 * There is no reference oracle for these: parity is against this restatement only.
 * ---------------------------------------------------------------------------- */
#define ORC_REF_SLOTS 25
#define ORC_MAXN 256
#define ORC_MAXSLOTS (ORC_MAXT + 1)

/* triple32 integer hash and the stream key shared with the GPU generator
 * (smart-nanogrid-gym_amd/csrc/sng_kernels.hip: mix32, stream_key). */
static uint32_t mix32(uint32_t x) {
    x ^= x >> 17; x *= 0xed5ad4bbu;
    x ^= x >> 11; x *= 0xac4c1b51u;
    x ^= x >> 15; x *= 0x31848babu;
    x ^= x >> 14;
    return x;
}

static uint32_t stream_key(uint64_t seed, uint64_t ge, uint32_t lane, uint64_t day) {
    uint32_t k0 = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + (uint32_t)day * 0x9e3779b9u));
    uint32_t k1 = mix32(k0 ^ (uint32_t)ge);
    return mix32(k1 ^ ((uint32_t)(ge >> 32) * 0x85ebca6bu + lane * 0xc2b2ae35u + 0x27d4eb2fu));
}

#define ORC_DOMAIN_PV 0x50560000u
#define ORC_DOMAIN_PRICE 0x50520000u

/* profile factor 1 + sigma * z, z = h * 2^-31 - 1 in [-1, 1) */
static double profile_factor(uint64_t env_seed, uint32_t domain, uint64_t day, int k, double sigma) {
    uint32_t key = stream_key(env_seed, 0, domain, day);
    uint32_t h = mix32(key + (uint32_t)k * 0x9e3779b9u);
    double z = (double)h * 0x1.0p-31 - 1.0;
    return 1.0 + sigma * z;
}

/* ------------------------------------------------------------------------------
 * Configuration and constant tables
 * ---------------------------------------------------------------------------- */
enum { PEN_NONE = 0, PEN_ON_DEPARTURE = 1, PEN_SPARSE = 2, PEN_DENSE = 3, PEN_INVALID = 4 };

typedef struct {
    int n_chargers;          /* number_of_chargers */
    int T;                   /* int(24 / dt) */
    double dt;               /* set_time_interval, smart_nanogrid_environment.py:125-138 */
    int pv, bess, v2x;
    int diff_caps;           /* enable_different_vehicle_battery_capacities */
    int req_enabled;         /* enable_requested_state_of_charge */
    int penalty_mode;        /* charging_station.py:50-60 */
    int bounded;             /* charging_mode == 'bounded' */
    int numpy_legacy;        /* 1: NumPy<2 promotion (action*22*0.95 in f64) */
    double grid_cost_weight; /* accountant.py:35 (0.75 in v1; 0.8 in the recorded KATs) */
    int extended;            /* build-defined extended day (see above) */
    int slots;               /* per-charger array length: 25 (charger.py:16-19), T+1 when extended */
    double pv_noise, price_noise;
    /* tables, built by orc_build_tables */
    int n_irr;
    double irr[4 * ORC_MAXT];       /* solar_irradiance_2[0, :], pv_system_manager.py:34-65 */
    double irr_max;
    double pv_power[4 * ORC_MAXT];  /* available_solar_power[0, :], :67-91 */
    int n_price;
    double price[4 * ORC_MAXT];     /* energy_price[0, :], accountant.py:48-101 (48 entries) */
    double price_max;
} orc_cfg;

/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h.src pairwise_sum):
 * what ndarray.sum()/mean() of a contiguous float64 run does. */
static double pairwise_sum(const double *a, long n) {
    if (n < 8) {
        double res = 0.0;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; j++) r[j] = a[j];
        long i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
    }
}

double orc_pairwise_sum(const double *a, long n) { return pairwise_sum(a, n); }

/* PVSystemManager (pv_system_manager.py:10-91) + Accountant (accountant.py:17-101).
 * Returns 0, or -1 for a price model the reference cannot build. */
int orc_build_tables(orc_cfg *c, int price_model, const double *irr_min, long n_min) {
    int T = c->T;
    int steps_min = (int)(60 * c->dt);                 /* pv_system_manager.py:35 */
    int padded = T * 2;                                /* 1 prediction day + 1 padding day, :11-15 */
    c->n_irr = padded;
    for (int k = 0; k < padded; k++) {
        long lo = (long)k * steps_min, hi = lo + steps_min;
        if (hi > n_min) hi = n_min;
        long cnt = hi - lo;
        c->irr[k] = cnt > 0 ? pairwise_sum(irr_min + lo, cnt) / (double)cnt : NAN;  /* mean(), :42 */
    }
    double mx = 0.0;                                   /* max(where >= 0, initial=0), :20 */
    for (int k = 0; k < padded; k++) if (c->irr[k] >= 0 && c->irr[k] > mx) mx = c->irr[k];
    c->irr_max = mx;
    double scaling_pv = ((2.279 * 1.134) * 20) * 0.21 / 1000;   /* :17, :72-73 */
    for (int k = 0; k < padded; k++)
        c->pv_power[k] = ((c->irr[k] * scaling_pv) * 1.5) / c->dt;  /* :67-70, :87-88 */

    double high = (0.028 + 0.148933333) + 0.014;       /* set_grid_tariffs, accountant.py:17-24 */
    double low = (0.013333333 + 0.087613333) + 0.014;
    static const double m1[24] = {0.05, 0.05, 0.05, 0.05, 0.05, 0.05, 0.05, 0.1, 0.1, 0.1, 0.1, 0.1,
                                  0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.1, 0.05, 0.05, 0.05, 0.05};
    static const double m2[24] = {0.05, 0.05, 0.05, 0.05, 0.05, 0.06, 0.07, 0.08, 0.09, 0.1, 0.1, 0.1,
                                  0.08, 0.06, 0.05, 0.05, 0.05, 0.06, 0.06, 0.06, 0.06, 0.05, 0.05, 0.05};
    static const double m3[24] = {0.071, 0.060, 0.056, 0.056, 0.056, 0.060, 0.060, 0.060, 0.066, 0.066, 0.076, 0.080,
                                  0.080, 0.1, 0.1, 0.076, 0.076, 0.1, 0.082, 0.080, 0.085, 0.079, 0.086, 0.070};
    static const double m4[24] = {0.1, 0.1, 0.05, 0.05, 0.05, 0.05, 0.05, 0.08, 0.08, 0.1, 0.1, 0.1,
                                  0.1, 0.1, 0.1, 0.1, 0.1, 0.06, 0.06, 0.06, 0.1, 0.1, 0.1, 0.1};
    double day[24];
    switch (price_model) {
        case 0: for (int h = 0; h < 24; h++) day[h] = (h < 7 || h >= 20) ? low : high; break; /* :69-73 */
        case 1: memcpy(day, m1, sizeof day); break;
        case 2: memcpy(day, m2, sizeof day); break;
        case 3: memcpy(day, m3, sizeof day); break;
        case 4: memcpy(day, m4, sizeof day); break;
        default: return -1;   /* model 5 raises TypeError (:90-98), others a shape error */
    }
    if (!c->extended) {
        c->n_price = 48;
        for (int k = 0; k < 48; k++) c->price[k] = day[k % 24];   /* concatenate twice, :100 */
    } else {
        /* per-step tariffs: the loop of accountant.py:61-68 for model 0, the hourly value otherwise */
        c->n_price = 2 * T;
        for (int i = 0; i < T; i++) {
            double v;
            if (price_model == 0) v = (i < 7 / c->dt || i > 19 / c->dt) ? low : high;
            else v = day[(int)floor(i * c->dt) % 24];
            c->price[i] = v;
            c->price[i + T] = v;
        }
    }
    mx = 0.0;
    for (int k = 0; k < c->n_price; k++) if (c->price[k] >= 0 && c->price[k] > mx) mx = c->price[k];
    c->price_max = mx;                                   /* accountant.py:51 */
    return 0;
}

/* ------------------------------------------------------------------------------
 * One environment, in the reference's own data structures
 * ---------------------------------------------------------------------------- */
typedef struct {
    double *soc, *cap, *occ, *req;              /* charger.py:16-19, cfg->slots entries each */
    int arrivals[ORC_MAXV], n_arr;              /* charger.vehicle_arrivals */
    int departures[ORC_MAXV], n_dep;            /* ChargingStation.departures[c] */
    double nonexistent;                         /* charger.py:146-156 */
} orc_charger;

typedef struct {
    const orc_cfg *cfg;
    orc_mt np_rng, py_rng;          /* global numpy / python RNG streams */
    uint64_t seed;                  /* this env's seed (profile noise key) */
    uint64_t day;                   /* resets so far (profile noise key) */
    int t;
    double ratio;                   /* random_pv_shift_ratio */
    double bess_soc, bess_init;     /* battery_energy_storage_system.py:6-22, initial 0.5 */
    double bess_power, bess_calc_power;
    int penalty_list[ORC_MAXN], n_penalty;  /* ChargingStation._penalty_check_vehicles */
    double f_pv[ORC_MAXT + 4], f_price[ORC_MAXT + 4];   /* this day's profile factors */
    orc_charger *ch;
    double *slotbuf;
    /* the last generated day, as initial_values.json holds it (charging_station.py:185-186) */
    orc_charger *gen;
    double *gen_slotbuf;
    int has_gen;
} orc_env;

/* Step record (the 28-key results dict subset the parity tests compare). */
typedef struct {
    double reward, grid_power, p_charge, p_discharge, bess_soc, pen_vehicle, pen_battery;
    double grid_cost, total_cost, solar_power, bess_power, bess_calc_power, nonexistent, bess_initial_soc;
    int done, breakpoint, error;   /* error: 1 = ValueError negative demand (central_management_system.py:158-159),
                                      2 = ValueError charging mode, 3 = ValueError BESS SoC > 1 */
} orc_step_out;

static int slot_index(const orc_cfg *c, int t) { return t < 0 ? c->slots + t : t; }   /* python negative index */

static int in_list(const int *l, int n, int v) {
    for (int i = 0; i < n; i++) if (l[i] == v) return 1;
    return 0;
}

static void charger_clear(orc_env *e, orc_charger *ch) {
    int S = e->cfg->slots;
    memset(ch->soc, 0, sizeof(double) * S); memset(ch->cap, 0, sizeof(double) * S);
    memset(ch->occ, 0, sizeof(double) * S); memset(ch->req, 0, sizeof(double) * S);
    ch->n_arr = ch->n_dep = 0;
    ch->nonexistent = 0.0;
}

orc_env *orc_env_new(const orc_cfg *c, uint64_t seed) {
    if (!c->extended && c->T > ORC_REF_SLOTS - 1) return NULL;   /* IndexError in the reference */
    orc_env *e = (orc_env *)calloc(1, sizeof(orc_env));
    if (!e) return NULL;
    e->cfg = c;
    e->ch = (orc_charger *)calloc((size_t)c->n_chargers, sizeof(orc_charger));
    e->slotbuf = (double *)calloc((size_t)c->n_chargers * 4 * c->slots, sizeof(double));
    e->gen = (orc_charger *)calloc((size_t)c->n_chargers, sizeof(orc_charger));
    e->gen_slotbuf = (double *)calloc((size_t)c->n_chargers * 4 * c->slots, sizeof(double));
    if (!e->ch || !e->slotbuf || !e->gen || !e->gen_slotbuf) {
        free(e->ch); free(e->slotbuf); free(e->gen); free(e->gen_slotbuf); free(e);
        return NULL;
    }
    for (int i = 0; i < c->n_chargers; i++) {
        double *b = e->slotbuf + (size_t)i * 4 * c->slots;
        e->ch[i].soc = b; e->ch[i].cap = b + c->slots; e->ch[i].occ = b + 2 * c->slots; e->ch[i].req = b + 3 * c->slots;
        double *g = e->gen_slotbuf + (size_t)i * 4 * c->slots;
        e->gen[i].soc = g; e->gen[i].cap = g + c->slots; e->gen[i].occ = g + 2 * c->slots; e->gen[i].req = g + 3 * c->slots;
    }
    orc_np_seed(&e->np_rng, (uint32_t)seed);
    orc_py_seed(&e->py_rng, seed);
    e->seed = seed;
    e->day = 0;
    e->bess_soc = 0.5;     /* central_management_system.py:35 */
    e->bess_init = 0.5;
    e->ratio = 1.0;        /* smart_nanogrid_environment.py:65 */
    return e;
}

void orc_env_free(orc_env *e) {
    if (!e) return;
    free(e->ch);
    free(e->slotbuf);
    free(e->gen);
    free(e->gen_slotbuf);
    free(e);
}

/* copy one charger's day (slot arrays and arrival/departure lists) */
static void charger_copy(int S, orc_charger *dst, const orc_charger *src) {
    memcpy(dst->soc, src->soc, sizeof(double) * S); memcpy(dst->cap, src->cap, sizeof(double) * S);
    memcpy(dst->occ, src->occ, sizeof(double) * S); memcpy(dst->req, src->req, sizeof(double) * S);
    memcpy(dst->arrivals, src->arrivals, sizeof dst->arrivals); dst->n_arr = src->n_arr;
    memcpy(dst->departures, src->departures, sizeof dst->departures); dst->n_dep = src->n_dep;
    dst->nonexistent = src->nonexistent;
}

/* The day's profile factors (build-defined; all 1.0 when both sigmas are 0). */
static void draw_profiles(orc_env *e) {
    const orc_cfg *c = e->cfg;
    for (int k = 0; k < c->T + 3; k++) {
        e->f_pv[k] = c->pv_noise != 0.0 ? profile_factor(e->seed, ORC_DOMAIN_PV, e->day, k, c->pv_noise) : 1.0;
        e->f_price[k] = c->price_noise != 0.0 ? profile_factor(e->seed, ORC_DOMAIN_PRICE, e->day, k, c->price_noise) : 1.0;
    }
    e->day += 1;
}

/* ChargingStation.generate_random_vehicle_departure_time, charging_station.py:271-279 */
static int gen_departure(orc_env *e, int t) {
    const orc_cfg *c = e->cfg;
    int total = c->T;
    int max_charging = t + (int)(10 / c->dt);
    int max_departing = total + (int)(1 / c->dt);
    int upper = max_charging < max_departing ? max_charging : max_departing;
    int low = t + (int)(4 / c->dt);
    int high = upper;
    if (low >= high) return low;
    return (int)orc_np_randint(&e->np_rng, low, high);
}

/* generate_random_requested_end_vehicle_state_of_charge, charging_station.py:261-265 */
static double gen_requested(orc_env *e, double arrival_soc) {
    double lo = arrival_soc <= 0.9 ? arrival_soc + 0.1 : 1.0;
    return orc_np_uniform(&e->np_rng, lo, 1.0);
}

/* generate_initial_vehicle_presence_per_charger, charging_station.py:200-255 */
static void gen_charger(orc_env *e, orc_charger *ch) {
    const orc_cfg *c = e->cfg;
    int present = 0, dep = 0, cap_gen = 0, req_gen = 0;
    double cur_cap = 0, cur_req = 0;
    int total = c->T;
    for (int t = 0; t < total; t++) {
        if (!present) {
            double r = orc_np_random(&e->np_rng);
            if ((r - 0.1) > 0.5 && t < total) {          /* round(rand() - 0.1) == 1, :214-215 */
                present = 1;
                ch->soc[t] = orc_np_uniform(&e->np_rng, 0.1, 0.9);     /* :257-259 */
                (void)gen_requested(e, ch->soc[t]);                     /* discarded draw, :219 */
                if (c->diff_caps && !cap_gen) {
                    cur_cap = (double)orc_np_randint(&e->np_rng, 15, 120);  /* :267-269 */
                    cap_gen = 1;
                } else if (!c->diff_caps && !cap_gen) {
                    cur_cap = 40; cap_gen = 1;
                }
                if (c->req_enabled && !req_gen) {
                    cur_req = gen_requested(e, ch->soc[t]); req_gen = 1;
                } else if (!c->req_enabled && !req_gen) {
                    cur_req = 1.0; req_gen = 1;
                }
                ch->arrivals[ch->n_arr++] = t;
                dep = gen_departure(e, t);
                ch->departures[ch->n_dep++] = dep;
            }
        }
        if (present && t < dep) {
            ch->occ[t] = 1; ch->cap[t] = cur_cap; ch->req[t] = cur_req;
        } else {
            present = 0;
            ch->occ[t] = 0; ch->cap[t] = 0; cap_gen = 0; cur_cap = 0.0;
            ch->req[t] = 0; cur_req = 0; req_gen = 0;
        }
    }
}

/* find_vehicles_for_penalty_check, charging_station.py:42-63 (+ :79-90) */
static void penalty_check(orc_env *e, int t) {
    const orc_cfg *c = e->cfg;
    if (t >= c->T) return;   /* returns [] without clearing, :43-44 */
    e->n_penalty = 0;
    for (int i = 0; i < c->n_chargers; i++) {
        orc_charger *ch = &e->ch[i];
        int allowed = 0;
        switch (c->penalty_mode) {
            case PEN_NONE: allowed = 0; break;
            case PEN_ON_DEPARTURE: allowed = in_list(ch->departures, ch->n_dep, t + 1); break;
            case PEN_SPARSE: allowed = in_list(ch->departures, ch->n_dep, t + 1) ||
                                       in_list(ch->departures, ch->n_dep, t + 2) ||
                                       in_list(ch->departures, ch->n_dep, t + 3); break;
            case PEN_DENSE: allowed = 1; break;
        }
        if (ch->occ[t] != 0 && allowed) e->penalty_list[e->n_penalty++] = i;
    }
}

/* CentralManagementSystem.observe + SmartNanogridEnv.__get_observations
 * (central_management_system.py:45-78, smart_nanogrid_environment.py:190-231) */
static int observe(orc_env *e, float *obs) {
    const orc_cfg *c = e->cfg;
    int t = e->t, N = c->n_chargers, k = 0;
    penalty_check(e, t);
    if (c->pv) obs[k++] = (float)(((c->irr[t] / c->irr_max) * e->ratio) * e->f_pv[t]);
    obs[k++] = (float)((c->price[t] / c->price_max) * e->f_price[t]);
    if (c->pv)
        for (int j = t + 1; j < t + 4 && j < c->n_irr; j++)
            obs[k++] = (float)(((c->irr[j] / c->irr_max) * e->ratio) * e->f_pv[j]);
    for (int j = t + 1; j < t + 4 && j < c->n_price; j++)
        obs[k++] = (float)((c->price[j] / c->price_max) * e->f_price[j]);
    for (int i = 0; i < N; i++) obs[k++] = (float)e->ch[i].soc[t];   /* extract_current_state_of_charge, :114-117 */
    for (int i = 0; i < N; i++) {                                      /* calculate_departure_times, :92-112 */
        orc_charger *ch = &e->ch[i];
        double d = 0;
        if (ch->occ[t] != 0) {
            for (int v = 0; v < ch->n_dep; v++)
                if (t <= ch->departures[v]) { d = ch->departures[v] - t; break; }
        }
        obs[k++] = (float)(d / 24);
    }
    if (c->bess) obs[k++] = (float)e->bess_soc;
    return k;
}

/* ChargingStation.clear_initialisation_variables + generate_new_initial_values
 * (charging_station.py:138-186), then SmartNanogridEnv.reset (smart_nanogrid_environment.py:311-351). */
int orc_env_reset(orc_env *e, float *obs) {
    const orc_cfg *c = e->cfg;
    e->t = 0;
    for (int i = 0; i < c->n_chargers; i++) {
        charger_clear(e, &e->ch[i]);
        gen_charger(e, &e->ch[i]);
        charger_copy(c->slots, &e->gen[i], &e->ch[i]);   /* json.dump(initial_values.json), :185-186 */
    }
    e->has_gen = 1;
    e->ratio = (double)orc_py_randint(&e->py_rng, 0, 180) / 100;   /* :349 */
    draw_profiles(e);
    return observe(e, obs);
}

/* SmartNanogridEnv.reset(generate_new_initial_values=False) (smart_nanogrid_environment.py:311-357):
 * ChargingStation.load_initial_values (charging_station.py:119-136) clears the chargers
 * (clear_initialisation_variables, :138-150) and reads back what the last generation wrote to
 * initial_values.json (:185-186): arrivals, departures, SOC, occupancy and capacities -- but not
 * Requested_SOC, which stays 0.  Then a new PV ratio from the Python stream (:349); the numpy stream
 * and the BESS are untouched, the day's profile factors are kept.  Returns -1 when no day was
 * generated (the reference would read whatever file is on disk). */
int orc_env_replay(orc_env *e, float *obs) {
    const orc_cfg *c = e->cfg;
    if (!e->has_gen) return -1;
    e->t = 0;
    for (int i = 0; i < c->n_chargers; i++) {
        orc_charger *ch = &e->ch[i];
        charger_copy(c->slots, ch, &e->gen[i]);
        memset(ch->req, 0, sizeof(double) * c->slots);
        ch->nonexistent = 0.0;
    }
    e->ratio = (double)orc_py_randint(&e->py_rng, 0, 180) / 100;
    return observe(e, obs);
}

/* Injected scenario (for known-answer replays): per-charger slot arrays + lists. */
int orc_env_load(orc_env *e, const double *soc, const double *occ, const double *cap, const double *req,
                 const int *arrivals, const int *departures, int vmax, double ratio, float *obs) {
    const orc_cfg *c = e->cfg;
    int S = c->slots;
    e->t = 0;
    for (int i = 0; i < c->n_chargers; i++) {
        orc_charger *ch = &e->ch[i];
        charger_clear(e, ch);
        for (int s = 0; s < S; s++) {
            ch->soc[s] = soc[i * S + s]; ch->occ[s] = occ[i * S + s];
            ch->cap[s] = cap[i * S + s]; ch->req[s] = req[i * S + s];
        }
        for (int v = 0; v < vmax; v++) {
            if (arrivals[i * vmax + v] >= 0) ch->arrivals[ch->n_arr++] = arrivals[i * vmax + v];
            if (departures[i * vmax + v] >= 0) ch->departures[ch->n_dep++] = departures[i * vmax + v];
        }
    }
    e->ratio = ratio;
    draw_profiles(e);
    return observe(e, obs);
}

void orc_env_set_bess_soc(orc_env *e, double soc) { e->bess_soc = soc; }
double orc_env_get_bess_soc(const orc_env *e) { return e->bess_soc; }
void orc_env_set_ratio(orc_env *e, double r) { e->ratio = r; }
double orc_env_get_ratio(const orc_env *e) { return e->ratio; }

/* Charger.charge_or_discharge_vehicle / charge_vehicle / discharge_vehicle
 * (charger.py:37-56, 58-90, 108-140).  Returns the power (f64 array element). */
static double charger_step(orc_env *e, orc_charger *ch, float a, int t, int *err) {
    const orc_cfg *c = e->cfg;
    double dt = c->dt;
    int arrived = in_list(ch->arrivals, ch->n_arr, t);
    int prev = arrived ? t : slot_index(c, t - 1);
    double power;
    if (a == 0) {
        power = 0.0;
        ch->soc[t] = ch->soc[prev];
    } else if (!c->bounded) {
        *err = 2;
        power = 0.0;
    } else {
        double cap = ch->cap[prev], soc = ch->soc[prev];
        double p, change;
        if (c->numpy_legacy) {                     /* NumPy 1.x: np.float32 * int -> float64 */
            p = ((double)a * 22) * 0.95;
            change = (p * dt) / cap;
        } else {                                   /* NumPy 2 (NEP 50): float32 arithmetic */
            volatile float pf = (a * 22.0f) * 0.95f;
            volatile float pdt = pf * (float)dt;
            p = (double)pf;
            change = (double)pdt / cap;
        }
        double calc = soc + change;
        if (a > 0) {
            ch->soc[t] = (1.0 < calc) ? 1.0 : calc;          /* min(calc, 1.0), :86 */
            power = p;
        } else {
            /* over_discharging_flag = ceil(0.5 * (1 + sign(calc))) is 1 for calc >= 0 (:122) */
            if (calc >= 0) power = -((soc * cap) / dt);     /* :128-132 */
            else power = p;
            ch->soc[t] = (calc > 0.0) ? calc : 0.0;         /* max(0.0, calc), :136 */
        }
    }
    ch->nonexistent = 0.0;
    return power;
}

/* `x ** 2` in the reference is libm pow(x, 2.0) (CPython float_pow / numpy npy_pow), which on
 * glibc is not always the correctly rounded x*x (about 0.1 % of inputs differ by one ulp).
 * The call goes through a volatile pointer so the compiler cannot rewrite it to x*x.
 * orc_set_square_mode(1) switches to x*x, the arithmetic the GPU kernels use, so the
 * GPU can also be checked bit-for-bit against this oracle. */
static double (*volatile libm_pow)(double, double) = pow;
static int square_mode = 0;
void orc_set_square_mode(int m) { square_mode = m; }
static double square(double x) { return square_mode ? x * x : libm_pow(x, 2.0); }

/* Penaliser.penalise_state_of_charge_outside_margin, penaliser.py:71-87 (insufficient branch) */
static double vehicle_penalty(double req, double cur) {
    double lo = 0.05 * req;
    if (cur < req - lo) return square((req - cur) * 10);
    return 0.0;
}

/* SmartNanogridEnv.step -> CentralManagementSystem.manage_nanogrid
 * (smart_nanogrid_environment.py:140-188, central_management_system.py:84-185) */
int orc_env_step(orc_env *e, const float *actions, float *obs, orc_step_out *out) {
    const orc_cfg *c = e->cfg;
    int N = c->n_chargers, t = e->t;
    memset(out, 0, sizeof *out);
    double ba = c->bess ? (double)actions[N] : 0.0;                    /* :85-91 */
    if (t == 0 && c->bess) e->bess_init = e->bess_soc;                 /* :93-94 */

    /* simulate_vehicle_charging, charging_station.py:281-300 */
    double power[ORC_MAXN], pos[ORC_MAXN] = {0}, neg[ORC_MAXN] = {0};
    int npos = 0, nneg = 0, err = 0;
    for (int i = 0; i < N; i++) {
        orc_charger *ch = &e->ch[i];
        float a = actions[i];
        if (ch->occ[t] == 1) {
            power[i] = charger_step(e, ch, a, t, &err);
        } else {
            power[i] = 0;
            ch->nonexistent = (a != 0) ? 100 : 0.0;                    /* reset_info_values */
        }
    }
    for (int i = 0; i < N; i++) {
        if (power[i] < 0) neg[nneg++] = power[i];
        if (power[i] > 0) pos[npos++] = power[i];
    }
    double p_dis = pairwise_sum(neg, nneg), p_ch = pairwise_sum(pos, npos);

    /* penalise_charging_vehicles_outside_bounds, penaliser.py:39-57: the list comes from the
     * previous observe(); `timestep in arrivals` tests an int against a list of lists and is
     * always False, so SoC/requested SoC are read at python index t-1. */
    double nonexist = 0;
    for (int i = 0; i < N; i++) nonexist += e->ch[i].nonexistent;
    double pen_v = 0;
    for (int k = 0; k < e->n_penalty; k++) {
        orc_charger *ch = &e->ch[e->penalty_list[k]];
        int s = slot_index(c, t - 1);
        pen_v += vehicle_penalty(ch->req[s], ch->soc[s]);
    }

    double solar = c->pv ? (c->pv_power[t] * e->ratio) * e->f_pv[t] : 0;   /* :99-103 */
    double demand = p_ch + p_dis;                                       /* :105 */
    if (demand < 0 && !c->v2x) err = 1;                                 /* :158-159 */
    else if (demand < 0 && c->v2x) out->breakpoint = 1;                 /* :160-165 */
    double rem = demand - solar;                                        /* :167 */
    double pen_b = 0.0;
    if (c->bess) {                                                      /* battery_energy_storage_system.py:30-106 */
        if (ba == 0) {
            e->bess_power = 0.0; e->bess_calc_power = 0.0;
        } else if (!c->bounded) {
            err = 2;
        } else if (ba > 0) {
            double avail = -rem;
            double cp = (ba * 44) * 0.95;
            double calc = e->bess_soc + (cp * c->dt) / 80;
            e->bess_calc_power = cp;
            e->bess_soc = (1.0 < calc) ? 1.0 : calc;
            e->bess_power = cp;
            rem = -(avail - cp);
        } else {
            double dp = (ba * 44) * 0.95;
            double calc = e->bess_soc + (dp * c->dt) / 80;
            e->bess_calc_power = dp;
            if (calc < 0) dp = -((e->bess_soc * 80) / c->dt);          /* :82-94 */
            e->bess_soc = (calc > 0.0) ? calc : 0.0;
            e->bess_power = dp;
            rem = rem + dp;
        }
        /* DoD penalty (penaliser_old.py:98-104 semantics; penaliser.py:104-111) */
        if (e->bess_soc < 0.15) pen_b = square((0.15 - e->bess_soc) * 10);
        else if (e->bess_soc <= 1.0) pen_b = 0.0;
        else err = 3;
    }
    double grid = rem;
    double energy = grid * c->dt;                                       /* :107 */
    double price = c->price[t] * e->f_price[t];
    double cost = energy < 0 ? (energy * 0.8) * price : energy * price; /* accountant.py:26-32 */
    double total_pen = 0.8 * pen_b + pen_v;                             /* penaliser.py:177-181 */
    double total = c->grid_cost_weight * fabs(cost) + total_pen;        /* accountant.py:34-36 */

    out->reward = -total;
    out->grid_power = grid; out->p_charge = p_ch; out->p_discharge = p_dis;
    out->bess_soc = c->bess ? e->bess_soc : 0.0;
    out->pen_vehicle = pen_v; out->pen_battery = pen_b;
    out->grid_cost = cost; out->total_cost = total; out->solar_power = solar;
    out->bess_power = c->bess ? e->bess_power : 0.0;
    out->bess_calc_power = c->bess ? e->bess_calc_power : 0.0;
    out->nonexistent = nonexist;
    out->bess_initial_soc = c->bess ? e->bess_init : 0.0;
    out->error = err;

    observe(e, obs);                                                    /* smart_nanogrid_environment.py:173 */
    e->t = t + 1;
    if ((double)e->t == 24.0 / c->dt) {                                 /* :174-181, :233-237 */
        out->done = 1;
        e->t = 0;
        e->ratio = (double)orc_py_randint(&e->py_rng, 0, 180) / 100;
    }
    return err;
}

/* Batched driver used for the CPU baseline: E independent environments, each stepped
 * through `episodes` full days with actions[t][env][A]; returns the sum of rewards. */
double orc_run_batch(const orc_cfg *cfg, int64_t n_envs, uint64_t seed, int episodes,
                     const float *actions, int64_t act_stride_env, float *obs_scratch) {
    double acc = 0;
    orc_step_out out;
    int T = cfg->T;
    for (int64_t i = 0; i < n_envs; i++) {
        orc_env *e = orc_env_new(cfg, seed + (uint64_t)i);
        if (!e) return NAN;
        for (int ep = 0; ep < episodes; ep++) {
            orc_env_reset(e, obs_scratch);
            for (int t = 0; t < T; t++) {
                const float *a = actions + ((int64_t)t * n_envs + i) * act_stride_env;
                orc_env_step(e, a, obs_scratch, &out);
                acc += out.reward;
            }
        }
        orc_env_free(e);
    }
    return acc;
}

/* ------------------------------------------------------------------------------
 * Flat entry points for the ctypes wrapper (oracle/oracle.py)
 * ---------------------------------------------------------------------------- */
orc_cfg *orc_cfg_new(int n_chargers, double dt, int pv, int bess, int v2x, int diff_caps, int req_enabled,
                     int penalty_mode, int bounded, int numpy_legacy, double grid_cost_weight, int price_model,
                     const double *irr_min, long n_min, int extended, double pv_noise, double price_noise) {
    if (n_chargers < 1 || n_chargers > ORC_MAXN) return NULL;
    orc_cfg *c = (orc_cfg *)calloc(1, sizeof(orc_cfg));
    c->n_chargers = n_chargers;
    c->dt = dt;
    c->T = (int)(24 / dt);
    c->extended = extended;
    /* a standard config with T > 24 only builds tables (the reference's own tables exist for any dt,
     * its 25-slot arrays do not run); orc_env_new refuses it */
    if (c->T < 1 || c->T > ORC_MAXT) { free(c); return NULL; }
    c->slots = extended ? c->T + 1 : ORC_REF_SLOTS;
    c->pv_noise = pv_noise; c->price_noise = price_noise;
    c->pv = pv; c->bess = bess; c->v2x = v2x; c->diff_caps = diff_caps; c->req_enabled = req_enabled;
    c->penalty_mode = penalty_mode; c->bounded = bounded; c->numpy_legacy = numpy_legacy;
    c->grid_cost_weight = grid_cost_weight;
    if (orc_build_tables(c, price_model, irr_min, n_min) != 0) { free(c); return NULL; }
    return c;
}

void orc_cfg_free(orc_cfg *c) { free(c); }

int orc_cfg_slots(const orc_cfg *c) { return c->slots; }

int orc_cfg_tables(const orc_cfg *c, double *irr, double *irr_max, double *pv_power, double *price,
                   double *price_max) {
    memcpy(irr, c->irr, sizeof(double) * c->n_irr);
    memcpy(pv_power, c->pv_power, sizeof(double) * c->n_irr);
    memcpy(price, c->price, sizeof(double) * c->n_price);
    *irr_max = c->irr_max;
    *price_max = c->price_max;
    return c->n_irr;
}

int orc_env_t(const orc_env *e) { return e->t; }

/* out: reward, grid_power, p_charge, p_discharge, bess_soc, pen_vehicle, pen_battery, grid_cost,
 *      total_cost, solar_power, bess_power, bess_calc_power, nonexistent, bess_initial_soc
 * iout: done, breakpoint, error */
int orc_env_step_flat(orc_env *e, const float *actions, float *obs, double *out, int *iout) {
    orc_step_out s;
    int err = orc_env_step(e, actions, obs, &s);
    double v[14] = {s.reward, s.grid_power, s.p_charge, s.p_discharge, s.bess_soc, s.pen_vehicle,
                    s.pen_battery, s.grid_cost, s.total_cost, s.solar_power, s.bess_power,
                    s.bess_calc_power, s.nonexistent, s.bess_initial_soc};
    memcpy(out, v, sizeof v);
    iout[0] = s.done; iout[1] = s.breakpoint; iout[2] = s.error;
    return err;
}

/* Export the current scenario in the reference's layout (slot arrays, padded lists). */
void orc_env_get_scenario(const orc_env *e, double *soc, double *occ, double *cap, double *req,
                          int *arrivals, int *departures, int vmax) {
    int S = e->cfg->slots;
    for (int i = 0; i < e->cfg->n_chargers; i++) {
        const orc_charger *ch = &e->ch[i];
        memcpy(soc + i * S, ch->soc, sizeof(double) * S);
        memcpy(occ + i * S, ch->occ, sizeof(double) * S);
        memcpy(cap + i * S, ch->cap, sizeof(double) * S);
        memcpy(req + i * S, ch->req, sizeof(double) * S);
        for (int v = 0; v < vmax; v++) {
            arrivals[i * vmax + v] = v < ch->n_arr ? ch->arrivals[v] : -1;
            departures[i * vmax + v] = v < ch->n_dep ? ch->departures[v] : -1;
        }
    }
}

/* Profile factors of the current day, [T + 3] each (build-defined noise). */
void orc_env_get_profiles(const orc_env *e, double *f_pv, double *f_price) {
    memcpy(f_pv, e->f_pv, sizeof(double) * (e->cfg->T + 3));
    memcpy(f_price, e->f_price, sizeof(double) * (e->cfg->T + 3));
}

/* RNG probes for the draw-for-draw tests against numpy / Python's random. */
orc_mt *orc_rng_new(uint64_t seed, int python_style) {
    orc_mt *s = (orc_mt *)malloc(sizeof(orc_mt));
    if (python_style) orc_py_seed(s, seed); else orc_np_seed(s, (uint32_t)seed);
    return s;
}
void orc_rng_free(orc_mt *s) { free(s); }
uint32_t orc_rng_u32(orc_mt *s) { return mt_next(s); }
double orc_rng_random(orc_mt *s) { return orc_np_random(s); }
double orc_rng_uniform(orc_mt *s, double lo, double hi) { return orc_np_uniform(s, lo, hi); }
int64_t orc_rng_np_randint(orc_mt *s, int64_t lo, int64_t hi) { return orc_np_randint(s, lo, hi); }
int64_t orc_rng_py_randint(orc_mt *s, int64_t a, int64_t b) { return orc_py_randint(s, a, b); }
