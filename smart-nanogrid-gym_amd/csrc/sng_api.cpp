// sng_api.cpp -- host side of libsng.so: the C ABI declared in include/sng.h.
//
// Owns the per-handle device state, builds the constant tables, turns days in the
// reference's own layout (25-slot arrays + arrival/departure lists) into the packed
// per-charger-step words the step kernel reads, generates reference-exact days on host
// threads (MT19937 streams) while uploading them, replays the last generated day, saves and
// restores the whole simulation state, and captures whole days into hipGraphs.
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sng.h"
#include "sng_layout.h"
#include "sng_mt.h"

namespace sng {
hipError_t launch_step(const Params &p, const DeviceState &s, const InfoPtrs &info, const Tables &tab,
                       const float *act, float *obs,
                       double *reward, uint8_t *done, int64_t E, int t, int vec_io, hipStream_t stream,
                       hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
hipError_t launch_observe0(const Params &p, const DeviceState &s, float *obs, double *ep_return, int64_t E,
                           int vec_io, hipStream_t stream, int mode, int64_t replay, const RefStreams *ps = nullptr,
                           int py = 0);
hipError_t launch_generate(const Params &p, const DeviceState &s, uint64_t seed, int64_t E, int i4, int i10, int i1,
                           float *obs, double *ep_return, int vec_io,
                           hipStream_t stream, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
hipError_t launch_profiles(const Params &p, const DeviceState &s, int64_t E, hipStream_t stream);
hipError_t launch_bump_day(const DeviceState &s, hipStream_t stream);
hipError_t launch_probe_copy(const void *in, void *out, int64_t nr, int64_t nw, hipStream_t stream, hipEvent_t a,
                             hipEvent_t b);
hipError_t launch_ref_seed(const RefStreams &rs, uint64_t seed0, int64_t E, hipStream_t stream);
hipError_t launch_mt_prepare(const RefStreams &rs, int64_t E, hipStream_t stream);
hipError_t launch_ref_day(const Params &p, const DeviceState &s, const RefStreams &rs, int64_t E, int i4, int i10,
                          int i1, bool prepare, hipStream_t stream);
int step_lanes_supported(int n, int lanes);
int step_kernel_name(const Params &p, const InfoPtrs &info, char *buf, int len);
}  // namespace sng

using namespace sng;

namespace {

thread_local std::string g_create_error;


// numpy pairwise_sum (contiguous float64), used by ndarray.mean() in
// PVSystemManager.calculate_solar_irradiance_mean (pv_system_manager.py:34-44)
double pairwise_sum(const double *a, long n) {
    if (n < 8) {
        double res = 0.0;
        for (long i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = a[j];
        long i = 8;
        for (; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; ++j) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    long n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

struct HostTables {
    std::vector<double> irr, pv_power, price;
    double irr_max = 0, price_max = 0;
};

// PVSystemManager (pv_system_manager.py:10-91) and Accountant price tables (accountant.py:17-101)
bool build_tables(const SngConfig &c, int T, HostTables &tb, std::string &err) {
    const double dt = c.time_interval_hours;
    const int steps_min = (int)(60 * dt);
    const int padded = 2 * T;
    if ((int64_t)padded * steps_min > c.irradiance_minutes) {
        err = "irradiance data too short for two days at this time interval";
        return false;
    }
    tb.irr.assign(padded, 0.0);
    tb.pv_power.assign(padded, 0.0);
    for (int k = 0; k < padded; ++k)
        tb.irr[k] = pairwise_sum(c.irradiance_per_minute + (int64_t)k * steps_min, steps_min) / (double)steps_min;
    double mx = 0.0;
    for (double v : tb.irr)
        if (v >= 0 && v > mx) mx = v;
    tb.irr_max = mx;
    const double scaling_pv = ((2.279 * 1.134) * 20) * 0.21 / 1000;   // PVSystem(...), pv_system_manager.py:17, :72-73
    for (int k = 0; k < padded; ++k) tb.pv_power[k] = ((tb.irr[k] * scaling_pv) * 1.5) / dt;

    const double high = (0.028 + 0.148933333) + 0.014;   // set_grid_tariffs, accountant.py:17-24
    const double low = (0.013333333 + 0.087613333) + 0.014;
    static const double m1[24] = {0.05, 0.05, 0.05, 0.05, 0.05, 0.05, 0.05, 0.1, 0.1, 0.1, 0.1, 0.1,
                                  0.1,  0.1,  0.1,  0.1,  0.1,  0.1,  0.1,  0.1, 0.05, 0.05, 0.05, 0.05};
    static const double m2[24] = {0.05, 0.05, 0.05, 0.05, 0.05, 0.06, 0.07, 0.08, 0.09, 0.1,  0.1,  0.1,
                                  0.08, 0.06, 0.05, 0.05, 0.05, 0.06, 0.06, 0.06, 0.06, 0.05, 0.05, 0.05};
    static const double m3[24] = {0.071, 0.060, 0.056, 0.056, 0.056, 0.060, 0.060, 0.060, 0.066, 0.066, 0.076, 0.080,
                                  0.080, 0.1,   0.1,   0.076, 0.076, 0.1,   0.082, 0.080, 0.085, 0.079, 0.086, 0.070};
    static const double m4[24] = {0.1, 0.1, 0.05, 0.05, 0.05, 0.05, 0.05, 0.08, 0.08, 0.1,  0.1,  0.1,
                                  0.1, 0.1, 0.1,  0.1,  0.1,  0.06, 0.06, 0.06, 0.1,  0.1,  0.1,  0.1};
    double day[24];
    switch (c.price_model) {
        case 0:
            for (int h = 0; h < 24; ++h) day[h] = (h < 7 || h >= 20) ? low : high;   // accountant.py:69-73
            break;
        case 1: std::memcpy(day, m1, sizeof day); break;
        case 2: std::memcpy(day, m2, sizeof day); break;
        case 3: std::memcpy(day, m3, sizeof day); break;
        case 4: std::memcpy(day, m4, sizeof day); break;
        default:
            err = "price_model must be 0..4 (model 5 raises TypeError in accountant.py:90-98)";
            return false;
    }
    if (!c.extended_day) {
        tb.price.assign(kPriceLen, 0.0);
        for (int k = 0; k < kPriceLen; ++k) tb.price[k] = day[k % 24];   // concatenate([day, day]), accountant.py:100
    } else {
        // build-defined extended day: the per-step tariff loop of accountant.py:61-68 for model 0,
        // the hourly value of hour floor(i*dt) for models 1-4; concatenated twice
        tb.price.assign(2 * T, 0.0);
        for (int i = 0; i < T; ++i) {
            const double v = (c.price_model == 0) ? ((i < 7 / dt || i > 19 / dt) ? low : high)
                                                  : day[(int)std::floor(i * dt) % 24];
            tb.price[i] = v;
            tb.price[i + T] = v;
        }
    }
    mx = 0.0;
    for (double v : tb.price)
        if (v >= 0 && v > mx) mx = v;
    tb.price_max = mx;
    return true;
}

bool in_list(const int32_t *l, int n, int v) {
    for (int i = 0; i < n; ++i)
        if (l[i] == v) return true;
    return false;
}

int list_len(const int32_t *l, int V) {
    int n = 0;
    while (n < V && l[n] >= 0) ++n;
    return n;
}

// One day of one environment in the reference's layout.
struct DayView {
    double *soc, *occ, *cap, *req;   // [N][S]
    int32_t *arr, *dep;              // [N][V], -1 padded
    int V;
    int S;                           // slots per charger: 25 (charger.py:16-19), T+1 with extended_day
};

// ChargingStation.generate_initial_vehicle_presence_per_charger and the draws it makes
// (charging_station.py:200-279), clear_initialisation_variables first (:138-150).
bool generate_day(const SngConfig &c, int T, MT19937 &rng, DayView d) {
    const int N = c.number_of_chargers;
    const double dt = c.time_interval_hours;
    const int S = d.S;
    std::fill(d.soc, d.soc + N * S, 0.0);
    std::fill(d.occ, d.occ + N * S, 0.0);
    std::fill(d.cap, d.cap + N * S, 0.0);
    std::fill(d.req, d.req + N * S, 0.0);
    std::fill(d.arr, d.arr + N * d.V, -1);
    std::fill(d.dep, d.dep + N * d.V, -1);
    for (int ch = 0; ch < N; ++ch) {
        double *soc = d.soc + ch * S, *occ = d.occ + ch * S, *cap = d.cap + ch * S, *req = d.req + ch * S;
        int32_t *arr = d.arr + ch * d.V, *dep_l = d.dep + ch * d.V;
        int na = 0;
        bool present = false, cap_gen = false, req_gen = false;
        int dep = 0;
        double cur_cap = 0, cur_req = 0;
        for (int t = 0; t < T; ++t) {
            if (!present) {
                const double r = rng.random();
                if ((r - 0.1) > 0.5 && t < T) {   // round(random.rand() - 0.1) == 1, :214-215
                    present = true;
                    soc[t] = rng.uniform(0.1, 0.9);                              // :257-259
                    {                                                            // discarded draw, :219
                        const double lo = soc[t] <= 0.9 ? soc[t] + 0.1 : 1.0;
                        (void)rng.uniform(lo, 1.0);
                    }
                    if (c.different_vehicle_capacities && !cap_gen) {
                        cur_cap = (double)rng.randint(15, 120);                  // :267-269
                        cap_gen = true;
                    } else if (!c.different_vehicle_capacities && !cap_gen) {
                        cur_cap = 40;
                        cap_gen = true;
                    }
                    if (c.requested_state_of_charge && !req_gen) {
                        const double lo = soc[t] <= 0.9 ? soc[t] + 0.1 : 1.0;   // :261-265
                        cur_req = rng.uniform(lo, 1.0);
                        req_gen = true;
                    } else if (!c.requested_state_of_charge && !req_gen) {
                        cur_req = 1.0;
                        req_gen = true;
                    }
                    if (na >= d.V) return false;
                    arr[na] = t;
                    // generate_random_vehicle_departure_time, :271-279
                    const int max_charging = t + (int)(10 / dt);
                    const int max_departing = T + (int)(1 / dt);
                    const int high = std::min(max_charging, max_departing);
                    const int low = t + (int)(4 / dt);
                    dep = (low >= high) ? low : (int)rng.randint(low, high);
                    dep_l[na] = dep;
                    ++na;
                }
            }
            if (present && t < dep) {
                occ[t] = 1;
                cap[t] = cur_cap;
                req[t] = cur_req;
            } else {
                present = false;
                occ[t] = 0;
                cap[t] = 0;
                cap_gen = false;
                cur_cap = 0.0;
                req[t] = 0;
                cur_req = 0;
                req_gen = false;
            }
        }
    }
    return true;
}

// Membership test of find_vehicles_for_penalty_check (charging_station.py:42-63, 79-90)
// for the list built by observe(t).
bool penalty_window(int mode, const int32_t *deps, int nd, int t) {
    switch (mode) {
        case SNG_PENALTY_ON_DEPARTURE: return in_list(deps, nd, t + 1);
        case SNG_PENALTY_SPARSE:
            return in_list(deps, nd, t + 1) || in_list(deps, nd, t + 2) || in_list(deps, nd, t + 3);
        case SNG_PENALTY_DENSE: return true;
        default: return false;
    }
}

// Encode one env's day into the dense per-charger-step timeline (sng_layout.h).
// req_out may be null; need_req reports whether any penalised requested SoC differs from 1.0.
bool encode_day(const Params &p, int64_t E, int64_t e, const DayView &d, uint32_t *word, double *aux,
                double *req_out, double *pen0, bool *need_req, std::string &err) {
    const int N = p.n, T = p.T;
    double pen_t0 = 0.0;
    for (int c = 0; c < N; ++c) {
        const int S = d.S;
        const double *soc = d.soc + c * S, *occ = d.occ + c * S, *cap = d.cap + c * S, *req = d.req + c * S;
        const int32_t *arr = d.arr + c * d.V, *dep = d.dep + c * d.V;
        const int na = list_len(arr, d.V), nd = list_len(dep, d.V);
        for (int t = 0; t < T; ++t) {
            const double o = occ[t];
            if (o != 0.0 && o != 1.0) {
                err = "occupancy values must be 0 or 1";
                return false;
            }
            const bool occupied = (o == 1.0);
            const bool arrived = in_list(arr, na, t);
            const int prev = arrived ? t : (t >= 1 ? t - 1 : S - 1);   // python index t-1
            // SOC[prev] is the running value only when step t-1 wrote it (charger occupied at t-1)
            const bool running = !arrived && t >= 1 && occ[t - 1] == 1.0;
            uint32_t capv = 0, rem = 0;
            double a = 0.0;
            if (occupied) {
                const double cv = cap[prev];
                if (!(cv >= 1.0 && cv <= 255.0 && cv == std::floor(cv))) {
                    err = "vehicle capacities of occupied chargers must be integers in [1, 255]";
                    return false;
                }
                capv = (uint32_t)cv;
                if (t == 0 && !arrived) {
                    err = "charger occupied at t=0 without an arrival at t=0";
                    return false;
                }
                int found = -1;
                for (int v = 0; v < nd; ++v)
                    if (t <= dep[v]) {
                        found = dep[v] - t;
                        break;
                    }
                if (found < 0 || found > 255) {
                    err = "occupied charger without a departure time >= t (or > 255 steps ahead)";
                    return false;
                }
                rem = (uint32_t)found;
                a = running ? 0.0 : soc[prev];
            } else {
                a = soc[t];
            }
            bool pen = false;
            if (t >= 1 && occ[t - 1] != 0.0) pen = penalty_window(p.penalty_mode, dep, nd, t - 1);
            const size_t idx = ((size_t)t * N + c) * (size_t)E + (size_t)e;
            word[idx] = pack_word(occupied, !running, pen, capv, rem);
            aux[idx] = a;
            if (pen && req[t - 1] != 1.0) *need_req = true;
            // Requested_SOC[c, t-1]; slot 0 keeps Requested_SOC[c, T-1] (sng_layout.h)
            if (req_out) req_out[idx] = req[t >= 1 ? t - 1 : T - 1];
        }
        // penalty at t = 0 reads python index -1 (slot 24) of SOC / Requested_SOC (penaliser.py:59-69)
        if (occ[0] != 0.0 && penalty_window(p.penalty_mode, dep, nd, 0)) {
            const double rq = req[S - 1], cur = soc[S - 1];
            if (cur < rq - 0.05 * rq) {
                const double x = (rq - cur) * 10;
                pen_t0 += x * x;
            }
        }
    }
    *pen0 = pen_t0;
    return true;
}

// Host threads for the reference-RNG day generator and the scenario encoder: the CPUs this process
// may run on (sched_getaffinity), capped by SNG_HOST_THREADS or OMP_NUM_THREADS when set (a GPU box
// shows the whole machine's CPUs but gives one process a share of them).
int host_threads() {
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    for (const char *var : {"SNG_HOST_THREADS", "OMP_NUM_THREADS"}) {
        const char *v = std::getenv(var);
        if (v && std::atoi(v) > 0) {
            n = std::min(n, std::atoi(v));
            break;
        }
    }
    return std::max(1, std::min(n, 64));
}

// A process-wide pool of host worker threads, started on first use and kept for the life of the
// process (never destroyed, so no worker is joined or torn down during static destruction).  A reset
// of 65,536 envs draws the Python-stream PV ratios in ~0.1 ms of work per thread; starting 15 threads
// for every reset cost more than the work.
class HostPool {
  public:
    static HostPool &get() {
        static HostPool *pool = new HostPool();
        return *pool;
    }
    // run job(k) for k in [0, parts) on the pool plus the calling thread; returns when all are done
    void run(int parts, const std::function<void(int)> &job) {
        std::unique_lock<std::mutex> call(call_mu_);   // one parallel section at a time
        grow(parts - 1);
        {
            std::lock_guard<std::mutex> lk(mu_);
            job_ = &job;
            parts_ = parts;
            next_ = 1;   // part 0 is the caller's
            done_ = 0;
            ++gen_;
        }
        cv_.notify_all();
        job(0);
        int k;
        while ((k = claim()) >= 0) {
            job(k);
            std::lock_guard<std::mutex> lk(mu_);
            ++done_;   // parts 1 .. parts - 1 count as done, whoever ran them
        }
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_ == parts_ - 1; });
        job_ = nullptr;
    }

  private:
    int claim() {
        std::lock_guard<std::mutex> lk(mu_);
        return next_ < parts_ ? next_++ : -1;
    }
    void grow(int want) {
        while ((int)workers_.size() < want) workers_.push_back(new std::thread([this] { loop(); }));
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(int)> *job;
            int k;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return gen_ != seen && job_ && next_ < parts_; });
                seen = gen_;
                job = job_;
                k = next_++;
            }
            for (;;) {
                (*job)(k);
                std::lock_guard<std::mutex> lk(mu_);
                ++done_;
                if (done_ == parts_ - 1) done_cv_.notify_one();
                if (next_ >= parts_) break;
                k = next_++;
            }
        }
    }
    std::mutex call_mu_, mu_;
    std::condition_variable cv_, done_cv_;
    std::vector<std::thread *> workers_;
    const std::function<void(int)> *job_ = nullptr;
    int parts_ = 0, next_ = 0, done_ = 0;
    uint64_t gen_ = 0;
};

// fn(begin, end) over [0, n) in contiguous ranges on host_threads() threads of the pool (the calling
// thread takes a range too); serial below `grain` items per thread.
template <class Fn>
void parallel_ranges(int64_t n, int64_t grain, Fn &&fn) {
    const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / grain));
    if (nt <= 1) {
        fn((int64_t)0, n);
        return;
    }
    const int64_t per = (n + nt - 1) / nt;
    HostPool::get().run(nt, [&](int k) {
        const int64_t b = k * per, en = std::min(n, b + per);
        if (b < en) fn(b, en);
    });
}

// FNV-1a over a byte range (the checkpoint's configuration fingerprint)
uint64_t fnv1a(const void *data, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char *b = static_cast<const unsigned char *>(data);
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ull;
    }
    return h;
}

// The checkpoint's configuration fingerprint: every SngConfig field that changes the simulation, hashed
// field by field (the struct's padding and -0.0 vs 0.0 must not make an identical configuration differ
// across processes or bindings).  The irradiance enters through the tables, hashed next to it.
uint64_t config_fingerprint(const SngConfig &c) {
    uint64_t h = 1469598103934665603ull;
    auto i32 = [&h](int32_t v) { h = fnv1a(&v, sizeof v, h); };
    auto f64 = [&h](double v) {
        if (v == 0.0) v = 0.0;   // -0.0 -> 0.0
        h = fnv1a(&v, sizeof v, h);
    };
    i32(c.abi_version);
    i32(c.number_of_chargers);
    f64(c.time_interval_hours);
    i32(c.price_model);
    i32(c.pv_system_available);
    i32(c.battery_system_available);
    i32(c.vehicle_to_everything);
    i32(c.different_vehicle_capacities);
    i32(c.requested_state_of_charge);
    i32(c.charging_mode_bounded);
    i32(c.penalty_mode);
    i32(c.numpy_legacy_promotion);
    for (double v : {c.grid_cost_weight, c.battery_penalty_weight, c.selling_price_coefficient, c.bess_capacity_kwh,
                     c.bess_initial_soc, c.bess_max_charging_kw, c.bess_max_discharging_kw, c.bess_charging_efficiency,
                     c.bess_discharging_efficiency, c.bess_depth_of_discharge, c.ev_max_power_kw, c.ev_efficiency})
        f64(v);
    i32(c.extended_day);
    f64(c.pv_noise);
    f64(c.price_noise);
    return h;
}

}  // namespace

struct SngEnv {
    SngConfig cfg{};
    Params p{};
    HostTables tables;
    Tables host_tab{};                // what d_tables holds
    uint64_t cfg_hash = 0;            // configuration fingerprint (scalars + tables), checked by sng_set_state
    std::vector<double> irradiance;   // owned copy
    int device = 0;
    int64_t E = 0;
    uint64_t seed = 0;
    int t = -1;                       // -1: never reset; T: day finished
    bool day_finished = false;        // the reference's end-of-day Python draw (:181) is still owed
    int i4 = 0, i10 = 0, i1 = 0;
    int slots = kSlots;               // per-charger array length of scenarios (T+1 with extended_day)
    // the day reset(generate_new_initial_values=False) replays: the last day sng_reset generated
    // (the reference's initial_values.json, charging_station.py:185-186 / :119-136)
    int gen_mode = -1;                // -1: none yet; else the SngRngMode that generated it
    bool gen_loaded = false;          // its timeline is still the loaded one (no injected day since)
    uint64_t replays = 0;             // device-RNG replays so far: the replay ratio stream's counter
    DeviceState ds{};
    Tables *d_tables = nullptr;
    // host staging (pinned) for days built on the CPU
    uint32_t *h_word = nullptr;
    double *h_aux = nullptr, *h_req = nullptr, *h_ratio = nullptr, *h_pen0 = nullptr;
    hipEvent_t staging_done = nullptr;
    // reference RNG streams of every env (allocated on first use): numpy's on the device (RefStreams,
    // drawn by ref_day_kernel), Python's on the host (two or three draws a day)
    RefStreams rs{};
    bool np_seeded = false;
    // the next day's stream blocks are prepared (mt_prepare_kernel) on a side stream while a day is stepped;
    // every access to rs on a caller's stream first waits for prep_done
    hipStream_t prep_stream = nullptr;
    hipEvent_t prep_done = nullptr, day_drawn = nullptr;
    bool prep_launched = false;   // prep_done marks a prepare launched on prep_stream

    bool prepared = false;        // the next day's blocks are (being) prepared: no inline prepare
    RefStreams ps{};                  // Python's `random` stream of every env, on the device (py_ratio_lane in observe0_kernel)
    bool py_seeded = false;
    // sng_step_host's I/O block: the step kernel reads its actions from and writes its outputs to host memory
    // (mapped, coherent), so a host-driven step is one dispatch and one wait.  A/B (profiles/r06_single_env.log,
    // SmartNanogridEnv.step at N = 10): 21.7 us per call against 25.4 us staged through a device block with a
    // copy each way, and 34.2 us for round 5's torch copies; tools/io_latency.hip: 13.0 / 17.2 us in C
    char *hio = nullptr, *hio_dev = nullptr;
    size_t hio_bytes = 0;
    std::string err;

    size_t timeline() const { return (size_t)p.T * p.n * (size_t)E; }
};

// The Params fields that say how the loaded day is encoded and stepped; a steps-only graph
// captures them and may replay only over a day with the same key.
struct DayKey {
    int32_t packed, req_stream, req_zero, bump_day;
    bool operator==(const DayKey &o) const {
        return packed == o.packed && req_stream == o.req_stream && req_zero == o.req_zero && bump_day == o.bump_day;
    }
};
static DayKey day_key(const Params &p) { return DayKey{p.packed, p.req_stream, p.req_zero, p.bump_day}; }

struct SngGraph {
    SngEnv *env = nullptr;
    bool with_reset = false;
    DayKey key{};   // the loaded-day encoding the graph's steps were captured for
    // the stream keys baked into the captured kernels' arguments: the device days a reset graph draws
    // and the PV-ratio / profile streams are those of this seed and env offset
    uint64_t seed = 0;
    int64_t env_offset = 0;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

namespace {

int fail(SngEnv *env, int code, const std::string &msg) {
    if (env) env->err = msg; else g_create_error = msg;
    return code;
}

// The device generator keeps the day's vehicles of a charger plus an end sentinel in 8 LDS slots
// (sng_kernels.hip, kDayVehicles): a vehicle stays >= 4/dt steps and leaves one step empty, so a
// day has at most T / (4/dt + 1) + 1 vehicles, which must leave the sentinel's slot free.
bool device_rng_ok(const SngEnv *env) { return env->i4 >= 2 && env->p.T / (env->i4 + 1) + 1 <= 7; }

int hip_fail(SngEnv *env, hipError_t e, const char *what) {
    return fail(env, SNG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(env, expr)                                   \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail(env, _e, #expr); \
    } while (0)

bool aligned16(const void *ptr) { return ((uintptr_t)ptr & 15u) == 0; }

InfoPtrs info_ptrs(const SngInfo *i) {
    InfoPtrs o{};
    if (!i) return o;
    o.grid_power = i->grid_power;
    o.p_charge = i->total_charging_power;
    o.p_discharge = i->total_discharging_power;
    o.bess_soc = i->battery_state_of_charge;
    o.pen_vehicle = i->total_vehicle_penalty;
    o.pen_battery = i->total_battery_penalty;
    o.grid_cost = i->grid_energy_cost;
    o.total_cost = i->total_cost;
    o.solar = i->utilized_solar_energy;
    o.bess_power = i->battery_power_value;
    o.bess_calc_power = i->battery_calculated_power;
    o.nonexistent = i->nonexistent_vehicle_penalty;
    o.bess_initial = i->initial_battery_soc;
    o.flags = i->flags;
    o.episode_return = i->episode_return;
    o.charger_power = i->charger_power;
    o.vehicle_soc = i->vehicle_soc;
    o.flag_any = i->flag_summary;
    return o;
}

int ensure_req(SngEnv *env) {
    if (!env->ds.req) HIP_TRY(env, hipMalloc(&env->ds.req, env->timeline() * sizeof(double)));
    return SNG_OK;
}

int ensure_staging(SngEnv *env, bool with_req) {
    const size_t n = env->timeline();
    if (!env->h_word) {
        HIP_TRY(env, hipHostMalloc(&env->h_word, n * sizeof(uint32_t), hipHostMallocDefault));
        HIP_TRY(env, hipHostMalloc(&env->h_aux, n * sizeof(double), hipHostMallocDefault));
        HIP_TRY(env, hipHostMalloc(&env->h_ratio, env->E * sizeof(double), hipHostMallocDefault));
        HIP_TRY(env, hipHostMalloc(&env->h_pen0, env->E * sizeof(double), hipHostMallocDefault));
        HIP_TRY(env, hipEventCreateWithFlags(&env->staging_done, hipEventDisableTiming));
    }
    if (with_req && !env->h_req) HIP_TRY(env, hipHostMalloc(&env->h_req, n * sizeof(double), hipHostMallocDefault));
    // the previous upload must have drained before the staging buffers are rewritten
    HIP_TRY(env, hipEventSynchronize(env->staging_done));
    return SNG_OK;
}

// The reference's global RNG streams of every env, np.random.seed(s) and random.seed(s) with
// s = seed + global env index (SngRngMode SNG_RNG_REFERENCE), both on the device.  Python's is seeded on
// the host threads (CPython's init_by_array, sng_mt.h) and uploaded once into the RefStreams layout
// (block 0, position N: the first draw twists), then drawn by observe0_kernel (py_ratio_lane): random.randint(0, 180)
// for a reset's PV ratio, after the day-end draw the last step owes (smart_nanogrid_environment.py:181, 349).
int await_prepare(SngEnv *env, hipStream_t st);
// numpy's np.random.seed takes seeds in [0, 2^32): env i of a reference-RNG population is seeded
// seed + env offset + i, so the last env's seed must stay below 2^32 (mt_seed_kernel would wrap it).
int check_reference_seed(SngEnv *env) {
    const uint64_t last = env->seed + (uint64_t)env->p.env_offset + (uint64_t)(env->E - 1);
    if (env->seed >= (1ull << 32) || last >= (1ull << 32) || last < env->seed)
        return fail(env, SNG_ERR_INVALID_ARGUMENT,
                    "the reference's RNG streams (a reference-RNG day, or a PV ratio drawn for an injected or replayed "
                    "day): seed + env offset + env index must be < 2^32 (np.random.seed's range)");
    return SNG_OK;
}

int ensure_py_streams(SngEnv *env, hipStream_t st) {
    const size_t E = (size_t)env->E;
    if (int rc = check_reference_seed(env)) return rc;
    if (!env->ps.mt) {
        HIP_TRY(env, hipMalloc(&env->ps.mt, E * 2 * kMtN * sizeof(uint32_t)));
        HIP_TRY(env, hipMalloc(&env->ps.pos, E * sizeof(int32_t)));
    }
    if (env->py_seeded) return SNG_OK;
    int rc = await_prepare(env, st);   // no preparation may still be writing the streams
    if (rc) return rc;
    std::vector<uint32_t> words(E * kMtN);
    std::vector<int32_t> pos(E);
    const uint64_t s0 = env->seed + (uint64_t)env->p.env_offset;
    parallel_ranges(env->E, 1024, [&](int64_t b, int64_t en) {
        MT19937 m;
        uint32_t st_words[MT19937::kStateWords];
        for (int64_t i = b; i < en; ++i) {
            m.seed_python(s0 + (uint64_t)i);
            m.save(st_words);
            for (int k = 0; k < kMtN; ++k) words[(size_t)i * kMtN + k] = mt_temper_word(st_words[k]);   // RefStreams keep tempered words
            pos[i] = (int32_t)st_words[kMtN];   // block 0, mti = N
        }
    });
    HIP_TRY(env, hipMemcpy2DAsync(env->ps.mt, 2 * kMtN * sizeof(uint32_t), words.data(), kMtN * sizeof(uint32_t),
                                  kMtN * sizeof(uint32_t), E, hipMemcpyHostToDevice, st));
    HIP_TRY(env, hipMemcpyAsync(env->ps.pos, pos.data(), E * sizeof(int32_t), hipMemcpyHostToDevice, st));
    // the first twist by a wavefront per env now, not by py_ratio_lane at the first draw
    HIP_TRY(env, launch_mt_prepare(env->ps, env->E, st));
    HIP_TRY(env, hipStreamSynchronize(st));   // the host vectors go out of scope
    env->py_seeded = true;
    return SNG_OK;
}

// Orders `st` after the side stream's preparation of the streams (sng_reset), before st touches them.
int await_prepare(SngEnv *env, hipStream_t st) {
    if (env->prep_launched) HIP_TRY(env, hipStreamWaitEvent(st, env->prep_done, 0));
    return SNG_OK;
}

// ... and numpy's on the device (mt_seed_kernel), queued on `st`.
int ensure_np_streams(SngEnv *env, hipStream_t st) {
    if (int rc = check_reference_seed(env)) return rc;
    if (!env->rs.mt) {
        HIP_TRY(env, hipMalloc(&env->rs.mt, (size_t)env->E * 2 * kMtN * sizeof(uint32_t)));
        HIP_TRY(env, hipMalloc(&env->rs.pos, (size_t)env->E * sizeof(int32_t)));
    }
    if (!env->np_seeded) {
        int rc = await_prepare(env, st);
        if (rc) return rc;
        HIP_TRY(env, launch_ref_seed(env->rs, env->seed + (uint64_t)env->p.env_offset, env->E, st));
        env->np_seeded = true;
        env->prepared = false;   // fresh streams: the first day prepares its blocks inline
    }
    return SNG_OK;
}

// Per-thread scratch for one env's day in the reference layout.
struct DayScratch {
    std::vector<double> soc, occ, cap, req;
    std::vector<int32_t> arr, dep;
    DayView view(int N, int S, int V) {
        soc.assign((size_t)N * S, 0.0);
        occ.assign((size_t)N * S, 0.0);
        cap.assign((size_t)N * S, 0.0);
        req.assign((size_t)N * S, 0.0);
        arr.assign((size_t)N * V, -1);
        dep.assign((size_t)N * V, -1);
        return DayView{soc.data(), occ.data(), cap.data(), req.data(), arr.data(), dep.data(), V, S};
    }
};

// Build every env's day on host threads and upload it while the rest is still being built:
// workers take chunks of envs and encode them into the pinned [T][N][E] staging planes; as soon as
// chunk k (in order) is encoded, this thread enqueues its columns of the planes as one 2D copy per
// plane.  build(i, scratch, need_req, err) builds env i.  req_upload: the requested-SoC plane goes
// up with the chunks (1), after the last chunk if any env needs it (-1: decided by need_req), or
// not at all (0).  Returns SNG_OK or an error; *need_req_out reports whether any env needed it.
template <class Build>
int build_and_upload(SngEnv *env, int req_upload, hipStream_t st, bool *need_req_out, Build &&build) {
    const int64_t E = env->E;
    const int N = env->p.n, T = env->p.T;
    const size_t rows = (size_t)T * N;
    const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, E / 256));
    const int64_t chunk = std::max<int64_t>(256, (E + 4 * nt - 1) / (4 * nt));   // ~4 chunks per thread
    const int64_t nchunks = (E + chunk - 1) / chunk;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> state((size_t)nchunks, 0);   // 0 pending, 1 encoded, 2 failed
    std::vector<std::string> errs((size_t)nchunks);
    std::atomic<int64_t> next{0};
    std::atomic<bool> stop{false}, need_req{false};
    auto worker = [&]() {
        DayScratch scratch;
        for (;;) {
            const int64_t k = next.fetch_add(1);
            if (k >= nchunks) return;
            int st_k = 1;
            std::string e;
            bool nr = false;
            if (stop.load()) {
                st_k = 2;
                e = "cancelled";
            } else {
                const int64_t b = k * chunk, en = std::min(E, b + chunk);
                for (int64_t i = b; i < en; ++i)
                    if (!build(i, scratch, &nr, e)) {
                        st_k = 2;
                        stop.store(true);
                        break;
                    }
            }
            if (nr) need_req.store(true);
            {
                std::lock_guard<std::mutex> lk(mu);
                state[(size_t)k] = st_k;
                errs[(size_t)k] = e;
            }
            cv.notify_one();
        }
    };
    std::vector<std::thread> th;
    for (int w = 0; w < nt; ++w) th.emplace_back(worker);
    int rc = SNG_OK;
    std::string msg;
    for (int64_t k = 0; k < nchunks && rc == SNG_OK; ++k) {
        int st_k;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return state[(size_t)k] != 0; });
            st_k = state[(size_t)k];
            msg = errs[(size_t)k];
        }
        if (st_k != 1) {
            rc = SNG_ERR_INVALID_ARGUMENT;
            break;
        }
        const int64_t b = k * chunk, w = std::min(E, b + chunk) - b;
        hipError_t e = hipMemcpy2DAsync(env->ds.word + b, E * sizeof(uint32_t), env->h_word + b, E * sizeof(uint32_t),
                                        w * sizeof(uint32_t), rows, hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = hipMemcpy2DAsync(env->ds.aux + b, E * sizeof(double), env->h_aux + b, E * sizeof(double),
                                 w * sizeof(double), rows, hipMemcpyHostToDevice, st);
        if (e == hipSuccess && req_upload == 1)
            e = hipMemcpy2DAsync(env->ds.req + b, E * sizeof(double), env->h_req + b, E * sizeof(double),
                                 w * sizeof(double), rows, hipMemcpyHostToDevice, st);
        if (e != hipSuccess) {
            rc = SNG_ERR_HIP;
            msg = std::string("staged upload: ") + hipGetErrorString(e);
        }
    }
    stop.store(rc != SNG_OK);
    for (auto &x : th) x.join();
    if (rc != SNG_OK) return fail(env, rc, msg);
    *need_req_out = need_req.load();
    if (req_upload == -1 && *need_req_out) {
        int r = ensure_req(env);
        if (r) return r;
        HIP_TRY(env, hipMemcpyAsync(env->ds.req, env->h_req, env->timeline() * sizeof(double),
                                    hipMemcpyHostToDevice, st));
    }
    return SNG_OK;
}

// After the day's planes: the PV ratios and t = 0 penalties, then the t = 0 observation.  py_end / py_draw:
// the Python streams' owed day-end draw / the ratio drawn on the device (in observe0_kernel) over the upload.
int finish_host_day(SngEnv *env, bool req_stream, float *obs, hipStream_t st, int py_end, int py_draw) {
    HIP_TRY(env, hipMemcpyAsync(env->ds.ratio, env->h_ratio, env->E * sizeof(double), hipMemcpyHostToDevice, st));
    HIP_TRY(env, hipMemcpyAsync(env->ds.pen0, env->h_pen0, env->E * sizeof(double), hipMemcpyHostToDevice, st));
    if (py_end || py_draw) {   // the draws themselves run inside observe0_kernel below
        int rc = await_prepare(env, st);
        if (rc) return rc;
    }
    HIP_TRY(env, hipEventRecord(env->staging_done, st));
    env->p.req_stream = req_stream ? 1 : 0;
    env->p.packed = 0;   // word + f64 aux planes
    env->p.req_zero = 0;
    env->p.bump_day = 0;
    HIP_TRY(env, sng::launch_profiles(env->p, env->ds, env->E, st));
    HIP_TRY(env, sng::launch_observe0(env->p, env->ds, obs, nullptr, env->E, aligned16(obs) ? 1 : 0, st, OBS0_HOST, -1,
                                      &env->ps, (py_draw ? 1 : 0) | (py_end ? 2 : 0)));
    env->t = 0;
    env->day_finished = false;
    return SNG_OK;
}

hipStream_t as_stream(void *s) { return (hipStream_t)s; }

}  // namespace

extern "C" {

int32_t sng_abi_version(void) { return SNG_ABI_VERSION; }
#ifndef SNG_BUILD_ID
#define SNG_BUILD_ID "unversioned"   // built outside csrc/Makefile
#endif
const char *sng_build_id(void) { return SNG_BUILD_ID; }

void sng_config_defaults(SngConfig *c) {
    std::memset(c, 0, sizeof *c);
    c->abi_version = SNG_ABI_VERSION;
    c->number_of_chargers = 8;                 // smart_nanogrid_environment.py:32
    c->time_interval_hours = 1.0;              // :138
    c->price_model = 0;
    c->pv_system_available = 1;
    c->battery_system_available = 1;
    c->vehicle_to_everything = 0;
    c->different_vehicle_capacities = 1;
    c->requested_state_of_charge = 0;
    c->charging_mode_bounded = 1;
    c->penalty_mode = SNG_PENALTY_SPARSE;
    c->numpy_legacy_promotion = 0;
    c->grid_cost_weight = 0.75;                // accountant.py:35
    c->battery_penalty_weight = 0.8;           // penaliser.py:181
    c->selling_price_coefficient = 0.8;        // accountant.py:6
    c->bess_capacity_kwh = 80;                 // central_management_system.py:35
    c->bess_initial_soc = 0.5;
    c->bess_max_charging_kw = 44;
    c->bess_max_discharging_kw = 44;
    c->bess_charging_efficiency = 0.95;
    c->bess_discharging_efficiency = 0.95;
    c->bess_depth_of_discharge = 0.15;
    c->ev_max_power_kw = 22;                   // charger.py:20-23
    c->ev_efficiency = 0.95;
}

const char *sng_last_error(const SngEnv *env) { return env ? env->err.c_str() : g_create_error.c_str(); }

static int validate(const SngConfig *c, int *T_out, std::string &err) {
    if (!c) { err = "null config"; return SNG_ERR_INVALID_ARGUMENT; }
    if (c->abi_version != SNG_ABI_VERSION) { err = "SngConfig.abi_version mismatch"; return SNG_ERR_INVALID_ARGUMENT; }
    if (c->number_of_chargers < 1 || c->number_of_chargers > kMaxChargers) {
        err = "number_of_chargers must be in [1, 128]";
        return SNG_ERR_UNSUPPORTED;
    }
    const double dt = c->time_interval_hours;
    if (!(dt > 0)) { err = "Wrong time interval was provided"; return SNG_ERR_INVALID_ARGUMENT; }
    const double steps = 24.0 / dt;
    const int T = (int)steps;
    if ((double)T != steps) {
        err = "24h / time_interval must be an integer (the reference never ends the day otherwise)";
        return SNG_ERR_UNSUPPORTED;
    }
    if (T > 24 && !c->extended_day) {
        err = "time intervals below 1h are not runnable in the reference (25-slot arrays, charger.py:16-19); "
              "set extended_day for the build-defined extension";
        return SNG_ERR_UNSUPPORTED;
    }
    if (T > kMaxT) { err = "at most 128 steps per day"; return SNG_ERR_UNSUPPORTED; }
    if (!(c->pv_noise >= 0.0 && c->pv_noise <= 1.0) || !(c->price_noise >= 0.0 && c->price_noise <= 1.0)) {
        err = "pv_noise / price_noise must be in [0, 1]";
        return SNG_ERR_INVALID_ARGUMENT;
    }
    if (T < 4) { err = "time interval too long (fewer than 4 steps per day)"; return SNG_ERR_UNSUPPORTED; }
    if (c->penalty_mode < 0 || c->penalty_mode > 3) {
        err = "Error: Wrong vehicle uncharged - penalty mode provided!";
        return SNG_ERR_INVALID_ARGUMENT;
    }
    if (c->price_model < 0 || c->price_model > 4) { err = "price_model must be 0..4"; return SNG_ERR_UNSUPPORTED; }
    if (!c->irradiance_per_minute || c->irradiance_minutes <= 0) {
        err = "irradiance_per_minute is required";
        return SNG_ERR_INVALID_ARGUMENT;
    }
    *T_out = T;
    return SNG_OK;
}

int sng_create(const SngConfig *cfg, int device, int64_t num_envs, uint64_t seed, SngEnv **out) {
    if (!out) return fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    int T = 0;
    std::string err;
    int rc = validate(cfg, &T, err);
    if (rc) return fail(nullptr, rc, err);
    if (num_envs < 1) return fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "num_envs must be >= 1");
    // the step kernel addresses a charger-major plane ([N][E] f64: the SoC state, one timestep of
    // the timeline) as one raw buffer with 32-bit byte offsets
    if ((uint64_t)num_envs * (uint64_t)cfg->number_of_chargers * sizeof(double) >= (1ull << 32))
        return fail(nullptr, SNG_ERR_INVALID_ARGUMENT,
                    "num_envs * number_of_chargers must be < 2^29 per handle (shard larger populations)");

    SngEnv *env = new SngEnv();
    env->cfg = *cfg;
    env->irradiance.assign(cfg->irradiance_per_minute, cfg->irradiance_per_minute + cfg->irradiance_minutes);
    env->cfg.irradiance_per_minute = env->irradiance.data();
    env->device = device;
    env->E = num_envs;
    env->seed = seed;
    if (!build_tables(env->cfg, T, env->tables, err)) {
        delete env;
        return fail(nullptr, SNG_ERR_UNSUPPORTED, err);
    }
    const SngConfig &c = env->cfg;
    Params &p = env->p;
    p.n = c.number_of_chargers;
    p.T = T;
    p.pv = c.pv_system_available ? 1 : 0;
    p.bess = c.battery_system_available ? 1 : 0;
    p.v2x = c.vehicle_to_everything ? 1 : 0;
    p.bounded = c.charging_mode_bounded ? 1 : 0;
    p.legacy = c.numpy_legacy_promotion ? 1 : 0;
    p.penalty_mode = c.penalty_mode;
    p.diff_caps = c.different_vehicle_capacities ? 1 : 0;
    p.req_enabled = c.requested_state_of_charge ? 1 : 0;
    p.req_stream = p.req_enabled;
    p.obs_dim = (1 + p.pv) * 4 + 2 * p.n + p.bess;   // smart_nanogrid_environment.py:90-96
    p.act_dim = p.n + p.bess;                          // :101-118
    p.dt = c.time_interval_hours;
    p.dt_f = (float)c.time_interval_hours;
    {
        int ex = 0;
        p.dt_pow2 = (std::frexp(p.dt, &ex) == 0.5) ? 1 : 0;   // dt = 2^k: x / dt == x * 2^-k
        p.rdt = 1.0 / p.dt;
    }
    p.ev_power = c.ev_max_power_kw;
    p.ev_eff = c.ev_efficiency;
    p.ev_power_f = (float)c.ev_max_power_kw;
    p.ev_eff_f = (float)c.ev_efficiency;
    p.bess_cap = c.bess_capacity_kwh;
    p.bess_pmax_ch = c.bess_max_charging_kw;
    p.bess_pmax_dis = c.bess_max_discharging_kw;
    p.bess_eff_ch = c.bess_charging_efficiency;
    p.bess_eff_dis = c.bess_discharging_efficiency;
    p.bess_dod = c.bess_depth_of_discharge;
    p.grid_w = c.grid_cost_weight;
    p.bat_pen_w = c.battery_penalty_weight;
    p.sell_coef = c.selling_price_coefficient;
    if (c.step_lanes_per_env) {
        if (!step_lanes_supported(p.n, c.step_lanes_per_env)) {
            delete env;
            return fail(nullptr, SNG_ERR_UNSUPPORTED, "step_lanes_per_env not available for this charger count");
        }
        p.lanes = c.step_lanes_per_env;
    } else {
        // tuned on MI355X at E=65,536 (bench.py --lanes): 1 lane per env at N=10 (7.6 / 8.9 / 11.4 us
        // for 1 / 2 / 4 lanes) and at N=50, config 5 (38.9 / 42.1 / 51.9 us)
        p.lanes = 1;
    }
    env->i4 = (int)(4 / p.dt);
    env->i10 = (int)(10 / p.dt);
    env->i1 = (int)(1 / p.dt);
    env->slots = c.extended_day ? T + 1 : kSlots;
    p.noise = (c.pv_noise > 0.0 || c.price_noise > 0.0) ? 1 : 0;
    p.pv_noise = c.pv_noise;
    p.price_noise = c.price_noise;
    p.seed = seed;

    // host copy of the device tables
    Tables &ht = env->host_tab;
    std::memset(&ht, 0, sizeof ht);
    const int n_irr = (int)env->tables.irr.size();
    ht.n_irr = n_irr;
    for (int k = 0; k < n_irr; ++k) {
        ht.irr_norm[k] = env->tables.irr[k] / env->tables.irr_max;   // pv_system_manager.py:81-85
        ht.pv_power[k] = env->tables.pv_power[k];
    }
    for (int k = 0; k < (int)env->tables.price.size(); ++k) {
        ht.price[k] = env->tables.price[k];
        ht.price_norm[k] = env->tables.price[k] / env->tables.price_max;   // accountant.py:42-46
    }
    ht.recip[0] = 0.0;
    for (int c = 1; c < 256; ++c) ht.recip[c] = 1.0 / (double)c;
    // checkpoint fingerprint: every configuration scalar that changes the simulation, and the tables
    env->cfg_hash = fnv1a(&ht, sizeof ht, config_fingerprint(c));

    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        delete env;
        return fail(nullptr, SNG_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
    }
    auto alloc = [&](void **ptr, size_t bytes) -> bool {
        hipError_t r = hipMalloc(ptr, bytes);
        if (r != hipSuccess) {
            g_create_error = std::string("hipMalloc: ") + hipGetErrorString(r);
            return false;
        }
        return true;
    };
    const size_t E = (size_t)num_envs, tl = env->timeline();
    DeviceState &ds = env->ds;
    bool ok = alloc((void **)&ds.soc, E * p.n * sizeof(double)) && alloc((void **)&ds.bess, E * sizeof(double)) &&
              alloc((void **)&ds.bess0, E * sizeof(double)) && alloc((void **)&ds.ratio, E * sizeof(double)) &&
              alloc((void **)&ds.pen0, E * sizeof(double)) && alloc((void **)&ds.word, tl * sizeof(uint32_t)) &&
              alloc((void **)&ds.aux, tl * sizeof(double)) && alloc((void **)&ds.flags, E * sizeof(uint32_t)) &&
              alloc((void **)&ds.episode, sizeof(uint64_t)) && alloc((void **)&env->d_tables, sizeof(Tables));
    if (ok && p.req_enabled) ok = alloc((void **)&ds.req, tl * sizeof(double));
    if (ok && p.noise) ok = alloc((void **)&ds.prof_key, 2 * (size_t)E * sizeof(uint32_t));
    if (!ok) {
        std::string msg = g_create_error;
        sng_destroy(env);
        return fail(nullptr, SNG_ERR_OUT_OF_MEMORY, msg);
    }
    ds.tables = env->d_tables;
    std::vector<double> b(E, c.bess_initial_soc);
    std::vector<double> ones(E, 1.0);
    bool ok2 = hipMemcpy(env->d_tables, &ht, sizeof ht, hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(ds.bess, b.data(), E * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(ds.bess0, b.data(), E * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
               hipMemcpy(ds.ratio, ones.data(), E * sizeof(double), hipMemcpyHostToDevice) == hipSuccess &&
               hipMemset(ds.pen0, 0, E * sizeof(double)) == hipSuccess &&
               hipMemset(ds.soc, 0, E * p.n * sizeof(double)) == hipSuccess &&
               hipMemset(ds.flags, 0, E * sizeof(uint32_t)) == hipSuccess &&
               hipMemset(ds.episode, 0, sizeof(uint64_t)) == hipSuccess &&
               hipMemset(ds.word, 0, tl * sizeof(uint32_t)) == hipSuccess &&
               hipMemset(ds.aux, 0, tl * sizeof(double)) == hipSuccess && hipDeviceSynchronize() == hipSuccess;
    if (!ok2) {
        sng_destroy(env);
        return fail(nullptr, SNG_ERR_HIP, "device initialisation failed");
    }
    *out = env;
    return SNG_OK;
}

void sng_destroy(SngEnv *env) {
    if (!env) return;
    (void)hipSetDevice(env->device);
    if (env->prep_stream) {
        (void)hipStreamSynchronize(env->prep_stream);
        (void)hipStreamDestroy(env->prep_stream);
        (void)hipEventDestroy(env->prep_done);
        (void)hipEventDestroy(env->day_drawn);
    }
    DeviceState &ds = env->ds;
    void *dev[] = {ds.soc, ds.bess, ds.bess0, ds.ratio, ds.pen0, ds.word, ds.aux, ds.req, ds.flags, ds.prof_key,
                   ds.episode, env->d_tables, env->rs.mt, env->rs.pos, env->ps.mt, env->ps.pos};
    for (void *x : dev)
        if (x) (void)hipFree(x);
    void *host[] = {env->h_word, env->h_aux, env->h_req, env->h_ratio, env->h_pen0};
    for (void *x : host)
        if (x) (void)hipHostFree(x);
    if (env->staging_done) (void)hipEventDestroy(env->staging_done);
    if (env->hio) (void)hipHostFree(env->hio);
    delete env;
}

int sng_get_dims(const SngEnv *env, SngDims *out) {
    if (!env || !out) return SNG_ERR_INVALID_ARGUMENT;
    out->obs_dim = env->p.obs_dim;
    out->act_dim = env->p.act_dim;
    out->timesteps = env->p.T;
    out->number_of_chargers = env->p.n;
    out->num_envs = env->E;
    out->step_lanes_per_env = env->p.lanes;
    out->slots = env->slots;
    return SNG_OK;
}

int sng_get_timestep(const SngEnv *env) { return env ? env->t : -1; }

int sng_set_env_offset(SngEnv *env, int64_t offset) {
    if (!env || offset < 0) return fail(env, SNG_ERR_INVALID_ARGUMENT, "bad env offset");
    env->p.env_offset = offset;
    env->np_seeded = false;   // reference streams are re-seeded (seed + offset + i) at the next reset
    env->py_seeded = false;
    env->day_finished = false;
    return SNG_OK;
}

int sng_set_seed(SngEnv *env, uint64_t seed, void *stream) {
    if (!env) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null handle");
    HIP_TRY(env, hipSetDevice(env->device));
    env->seed = seed;
    env->p.seed = seed;
    env->np_seeded = false;   // re-seeded (seed + offset + i) at the next reset
    env->py_seeded = false;
    env->day_finished = false;
    env->replays = 0;
    // device days restart at day 0 of the new streams; the loaded day stays loaded
    HIP_TRY(env, hipMemsetAsync(env->ds.episode, 0, sizeof(uint64_t), as_stream(stream)));
    if (env->p.packed && env->t == 0) env->p.bump_day = 0;   // an unstepped device day no longer owns day 0
    HIP_TRY(env, hipStreamSynchronize(as_stream(stream)));
    return SNG_OK;
}

int sng_reset(SngEnv *env, int rng_mode, float *obs, void *stream) {
    if (!env || !obs) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    if (rng_mode == SNG_RNG_DEVICE) {
        if (!device_rng_ok(env)) return fail(env, SNG_ERR_UNSUPPORTED, "device RNG needs time_interval <= 2h");
        const bool unstepped_device_day = env->p.packed && env->p.bump_day && env->t == 0;
        env->p.req_stream = env->p.req_enabled;
        env->p.packed = 1;   // the generator writes packed records (sng_layout.h)
        env->p.req_zero = 0;
        env->p.bump_day = 1;
        if (env->p.req_stream) {
            int rc = ensure_req(env);
            if (rc) return rc;
        }
        // a device day's first step advances the day counter (step_kernel); a second device reset
        // with no step in between advances it here, so it still draws a new day
        if (unstepped_device_day) HIP_TRY(env, launch_bump_day(env->ds, st));
        HIP_TRY(env, launch_generate(env->p, env->ds, env->seed, env->E, env->i4, env->i10, env->i1, obs, nullptr,
                                     aligned16(obs) ? 1 : 0, st));
        env->t = 0;
        env->day_finished = false;
        env->gen_mode = SNG_RNG_DEVICE;
        env->gen_loaded = true;
        return SNG_OK;
    }
    if (rng_mode != SNG_RNG_REFERENCE) return fail(env, SNG_ERR_INVALID_ARGUMENT, "unknown rng_mode");

    // the day on the device (ref_day2_kernel: numpy's stream, draw for draw), then the PV ratio from each
    // env's Python stream on the device, after the day-end draw the last step still owes
    // (smart_nanogrid_environment.py:181, 349)
    int rc = ensure_np_streams(env, st);
    if (rc) return rc;
    rc = ensure_py_streams(env, st);
    if (rc) return rc;
    const bool with_req = env->p.req_enabled != 0;
    if (with_req) {
        rc = ensure_req(env);
        if (rc) return rc;
    }
    rc = await_prepare(env, st);
    if (rc) return rc;
    if (!env->prep_stream) {
        HIP_TRY(env, hipStreamCreateWithFlags(&env->prep_stream, hipStreamNonBlocking));
        HIP_TRY(env, hipEventCreateWithFlags(&env->prep_done, hipEventDisableTiming));
        HIP_TRY(env, hipEventCreateWithFlags(&env->day_drawn, hipEventDisableTiming));
    }
    env->p.req_stream = with_req ? 1 : 0;
    HIP_TRY(env, launch_ref_day(env->p, env->ds, env->rs, env->E, env->i4, env->i10, env->i1, !env->prepared, st));
    env->p.packed = 0;   // word + f64 aux planes
    env->p.req_zero = 0;
    env->p.bump_day = 0;
    HIP_TRY(env, sng::launch_profiles(env->p, env->ds, env->E, st));
    // (the t = 0 penalty of a generated day is 0: observe0 writes it)
    // (the PV ratio from each env's Python stream, after the owed day-end draw, inside observe0_kernel)
    HIP_TRY(env, sng::launch_observe0(env->p, env->ds, obs, nullptr, env->E, aligned16(obs) ? 1 : 0, st, OBS0_GENERATED,
                                      -1, &env->ps, 1 | (env->day_finished ? 2 : 0)));
    // the next day's blocks of both streams, on the side stream, while this day is stepped
    // (mt_prepare_kernel: about every other day twists a numpy block, ~0.1 ms at 65,536 envs, off the next
    // reset's critical path); queued behind the t = 0 observation, which it would otherwise slow down
    HIP_TRY(env, hipEventRecord(env->day_drawn, st));
    HIP_TRY(env, hipStreamWaitEvent(env->prep_stream, env->day_drawn, 0));
    HIP_TRY(env, launch_mt_prepare(env->rs, env->E, env->prep_stream));
    HIP_TRY(env, launch_mt_prepare(env->ps, env->E, env->prep_stream));
    HIP_TRY(env, hipEventRecord(env->prep_done, env->prep_stream));
    env->prep_launched = true;
    env->prepared = true;
    env->t = 0;
    env->day_finished = false;
    env->gen_mode = SNG_RNG_REFERENCE;
    env->gen_loaded = true;
    return SNG_OK;
}

int sng_reset_replay(SngEnv *env, float *obs, void *stream) {
    if (!env || !obs) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (env->gen_mode < 0 || !env->gen_loaded)
        return fail(env, SNG_ERR_STATE,
                    env->gen_mode < 0 ? "reset(generate_new_initial_values=False) replays the last generated day "
                                        "(initial_values.json, charging_station.py:185-186): none was generated yet"
                                      : "reset(generate_new_initial_values=False) replays the last generated day; an "
                                        "injected day (sng_reset_from_scenario) has replaced it since");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    const int vec = aligned16(obs) ? 1 : 0;
    // a device day is counted by its first step; one replayed before any step was never counted, and
    // the replay's steps do not count (bump_day = 0 below), so count it here, as sng_reset does for a
    // second device reset in a row: the next device reset then draws a new day
    if (env->p.packed && env->p.bump_day && env->t == 0) HIP_TRY(env, launch_bump_day(env->ds, st));
    if (env->gen_mode == SNG_RNG_REFERENCE) {
        // a new random_pv_shift_ratio from each env's Python stream (smart_nanogrid_environment.py:349),
        // after the day-end draw the last step still owes (:181); the numpy stream is not touched
        int rc = ensure_py_streams(env, st);
        if (rc) return rc;
        rc = await_prepare(env, st);
        if (rc) return rc;
        env->p.req_zero = 1;
        env->p.bump_day = 0;
        HIP_TRY(env, sng::launch_observe0(env->p, env->ds, obs, nullptr, env->E, vec, st, OBS0_REPLAY, -1, &env->ps,
                                          1 | (env->day_finished ? 2 : 0)));
    } else {
        env->p.req_zero = 1;
        env->p.bump_day = 0;
        HIP_TRY(env, sng::launch_observe0(env->p, env->ds, obs, nullptr, env->E, vec, st, OBS0_REPLAY,
                                          (int64_t)env->replays));
        env->replays += 1;
    }
    env->t = 0;
    env->day_finished = false;
    return SNG_OK;
}

int sng_reset_from_scenario(SngEnv *env, const SngScenario *sc, float *obs, void *stream) {
    if (!env || !sc || !obs) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (sc->slots != env->slots)
        return fail(env, SNG_ERR_INVALID_ARGUMENT,
                    "scenario slots must be " + std::to_string(env->slots) + " (25; T+1 with extended_day)");
    if (!sc->soc || !sc->occupancy || !sc->capacity || !sc->requested_soc || !sc->arrivals || !sc->departures ||
        sc->max_vehicles < 1)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "incomplete scenario");
    HIP_TRY(env, hipSetDevice(env->device));
    int rc = ensure_staging(env, true);
    if (rc) return rc;
    // Python-stream accounting (env i == the reference seeded seed + i): the day-end draw the last
    // step still owes (smart_nanogrid_environment.py:181), and, when no ratio is given, the reset's own
    // draw (:349) -- what reset(generate_new_initial_values=False) consumes
    const bool draw_ratio = sc->pv_ratio == nullptr;
    if (draw_ratio) {
        rc = ensure_py_streams(env, as_stream(stream));
        if (rc) return rc;
    }
    const bool end_draw = env->day_finished && env->py_seeded;
    const int N = env->p.n, V = sc->max_vehicles, S = env->slots;
    // the requested-SoC plane goes up with the chunks when the config enables it (the step reads it
    // then), else only if some penalised slot of the given days is not 1.0
    const bool req_enabled = env->p.req_enabled != 0;
    if (req_enabled) {
        rc = ensure_req(env);
        if (rc) return rc;
    }
    bool need = false;
    rc = build_and_upload(env, req_enabled ? 1 : -1, as_stream(stream), &need,
                          [&](int64_t i, DayScratch &, bool *nr, std::string &e) -> bool {
                              const size_t o = (size_t)i * N * S, ol = (size_t)i * N * V;
                              DayView d{const_cast<double *>(sc->soc + o), const_cast<double *>(sc->occupancy + o),
                                        const_cast<double *>(sc->capacity + o),
                                        const_cast<double *>(sc->requested_soc + o),
                                        const_cast<int32_t *>(sc->arrivals + ol),
                                        const_cast<int32_t *>(sc->departures + ol), V, S};
                              env->h_ratio[i] = draw_ratio ? 1.0 : sc->pv_ratio[i];   // (drawn on the device)
                              if (!encode_day(env->p, env->E, i, d, env->h_word, env->h_aux, env->h_req,
                                              &env->h_pen0[i], nr, e)) {
                                  e = "env " + std::to_string(i) + ": " + e;
                                  return false;
                              }
                              return true;
                          });
    if (rc) {
        // chunks before the failing env are already uploaded over the loaded day's planes: the loaded
        // day is no longer valid, so step, replay and steps-only graphs refuse until the next reset (no
        // Python-stream draw was made)
        env->t = -1;
        env->gen_loaded = false;
        env->day_finished = false;
        env->err += " (the loaded day was partly overwritten: reset again)";
        return rc;
    }
    rc = finish_host_day(env, req_enabled || need, obs, as_stream(stream), end_draw ? 1 : 0, draw_ratio ? 1 : 0);
    if (rc) return rc;
    env->gen_loaded = false;   // the generated day a replay restores is no longer loaded
    return SNG_OK;
}

// The handle's device for the length of a call, the caller's current device restored after it (sng_step and
// sng_step_host are called per step without a device guard of the caller's own).
struct DeviceScope {
    int prev = -1, dev;
    hipError_t err = hipSuccess;
    explicit DeviceScope(int d) : dev(d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) err = hipSetDevice(d);
    }
    ~DeviceScope() {
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};

int sng_step(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done, const SngInfo *info,
             void *stream) {
    if (!env || !actions || !obs || !reward || !done) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (env->t < 0) return fail(env, SNG_ERR_STATE, "step() before reset()");
    if (env->t >= env->p.T) return fail(env, SNG_ERR_STATE, "the day is over: call reset()");
    DeviceScope dev(env->device);
    HIP_TRY(env, dev.err);
    const int vec = (aligned16(actions) && aligned16(obs)) ? 1 : 0;
    HIP_TRY(env, launch_step(env->p, env->ds, info_ptrs(info), env->host_tab, actions, obs, reward, done, env->E, env->t, vec,
                             as_stream(stream)));
    env->t += 1;
    if (env->t == env->p.T) env->day_finished = true;
    return SNG_OK;
}

int sng_step_host(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done, uint32_t *step_flags,
                  const SngInfo *info, void *stream) {
    if (!env || !actions || !obs || !reward || !done || !step_flags)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (env->t < 0) return fail(env, SNG_ERR_STATE, "step() before reset()");
    if (env->t >= env->p.T) return fail(env, SNG_ERR_STATE, "the day is over: call reset()");
    if (info && info->flags)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "sng_step_host returns the step's flags itself: SngInfo.flags must be null");
    DeviceScope dev(env->device);
    HIP_TRY(env, dev.err);
    hipStream_t st = as_stream(stream);
    const size_t E = (size_t)env->E, A = (size_t)env->p.act_dim, O = (size_t)env->p.obs_dim;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    // [actions E x A f32 | obs E x O f32 | reward E f64 | done E u8 | flags E u32], sections 256 B aligned
    const size_t o_obs = al(E * A * 4), o_rew = o_obs + al(E * O * 4), o_done = o_rew + al(E * 8),
                 o_fl = o_done + al(E), bytes = o_fl + al(E * 4);
    if (env->hio_bytes < bytes) {
        if (env->hio) (void)hipHostFree(env->hio);
        env->hio = env->hio_dev = nullptr;
        env->hio_bytes = 0;
        HIP_TRY(env, hipHostMalloc((void **)&env->hio, bytes, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(env, hipHostGetDevicePointer((void **)&env->hio_dev, env->hio, 0));
        env->hio_bytes = bytes;
    }
    char *h = env->hio, *d = env->hio_dev;
    std::memcpy(h, actions, E * A * 4);
    InfoPtrs ip = info_ptrs(info);
    ip.flags = reinterpret_cast<uint32_t *>(d + o_fl);   // this step's flags of every env (the sticky ones stay)
    HIP_TRY(env, launch_step(env->p, env->ds, ip, env->host_tab, reinterpret_cast<const float *>(d),
                             reinterpret_cast<float *>(d + o_obs), reinterpret_cast<double *>(d + o_rew),
                             reinterpret_cast<uint8_t *>(d + o_done), env->E, env->t, 1, st));
    env->t += 1;
    if (env->t == env->p.T) env->day_finished = true;
    HIP_TRY(env, hipStreamSynchronize(st));
    std::memcpy(obs, h + o_obs, E * O * 4);
    std::memcpy(reward, h + o_rew, E * 8);
    std::memcpy(done, h + o_done, E);
    std::memcpy(step_flags, h + o_fl, E * 4);
    return SNG_OK;
}

int sng_step_kernel_name(const SngEnv *env, const SngInfo *info, char *buf, int32_t len) {
    if (!env || !buf || len < 1) return SNG_ERR_INVALID_ARGUMENT;
    const int n = step_kernel_name(env->p, info_ptrs(info), buf, len);
    return (n > 0 && n < len) ? SNG_OK : SNG_ERR_INVALID_ARGUMENT;
}

int sng_read_errors(SngEnv *env, uint32_t *host_flags, int clear, void *stream) {
    if (!env || !host_flags) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    HIP_TRY(env, hipMemcpyAsync(host_flags, env->ds.flags, env->E * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    if (clear) HIP_TRY(env, hipMemsetAsync(env->ds.flags, 0, env->E * sizeof(uint32_t), st));
    HIP_TRY(env, hipStreamSynchronize(st));
    return SNG_OK;
}

// One per-env f64 array between the device and the host, ordered on `stream` (the caller's work on it
// completes first); synchronises that stream only.
static int copy_env_array(SngEnv *env, double *dev, double *host, bool to_host, void *stream, const char *what) {
    if (!env) return SNG_ERR_INVALID_ARGUMENT;
    if (!host) return fail(env, SNG_ERR_INVALID_ARGUMENT, std::string(what) + ": null host array");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    if (to_host)
        HIP_TRY(env, hipMemcpyAsync(host, dev, env->E * sizeof(double), hipMemcpyDeviceToHost, st));
    else
        HIP_TRY(env, hipMemcpyAsync(dev, host, env->E * sizeof(double), hipMemcpyHostToDevice, st));
    HIP_TRY(env, hipStreamSynchronize(st));
    return SNG_OK;
}

int sng_get_battery_soc(SngEnv *env, double *h, void *stream) {
    return env ? copy_env_array(env, env->ds.bess, h, true, stream, "sng_get_battery_soc") : SNG_ERR_INVALID_ARGUMENT;
}

int sng_set_battery_soc(SngEnv *env, const double *h, void *stream) {
    return env ? copy_env_array(env, env->ds.bess, const_cast<double *>(h), false, stream, "sng_set_battery_soc")
               : SNG_ERR_INVALID_ARGUMENT;
}

int sng_get_pv_ratio(SngEnv *env, double *h, void *stream) {
    return env ? copy_env_array(env, env->ds.ratio, h, true, stream, "sng_get_pv_ratio") : SNG_ERR_INVALID_ARGUMENT;
}

int sng_get_vehicle_soc(SngEnv *env, double *h, void *stream) {
    if (!env) return SNG_ERR_INVALID_ARGUMENT;
    if (!h) return fail(env, SNG_ERR_INVALID_ARGUMENT, "sng_get_vehicle_soc: null host array");
    HIP_TRY(env, hipSetDevice(env->device));
    const int N = env->p.n;
    hipStream_t st = as_stream(stream);
    // charger pairs on the device (sng_layout.h soc_index) -> [E][N] on the host
    std::vector<double> tmp((size_t)N * env->E);
    HIP_TRY(env, hipMemcpyAsync(tmp.data(), env->ds.soc, tmp.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    // a packed day: an empty charger's running SoC carries the next arrival's (sng_layout.h); SOC[c, t]
    // shows 0 there.  Occupancy of the last stepped step t - 1 is its record's OCC bit (plane t)
    std::vector<uint16_t> rec;
    const bool packed_mid = env->p.packed && env->t >= 1;
    if (packed_mid) {
        rec.resize((size_t)N * env->E);
        HIP_TRY(env, hipMemcpyAsync(rec.data(), reinterpret_cast<const uint16_t *>(env->ds.aux) + (size_t)env->t * rec.size(),
                                    rec.size() * sizeof(uint16_t), hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(env, hipStreamSynchronize(st));
    for (int64_t e = 0; e < env->E; ++e)
        for (int c = 0; c < N; ++c) {
            // the record plane in charger quads, the SoC state in charger pairs (sng_layout.h)
            h[e * N + c] = (packed_mid && !(rec[rec_index(c, e, N, env->E)] & W_OCC)) ? 0.0 : tmp[soc_index(c, e, N, env->E)];
        }
    return SNG_OK;
}

int sng_set_vehicle_soc(SngEnv *env, const double *h, void *stream) {
    if (!env) return SNG_ERR_INVALID_ARGUMENT;
    if (!h) return fail(env, SNG_ERR_INVALID_ARGUMENT, "sng_set_vehicle_soc: null host array");
    HIP_TRY(env, hipSetDevice(env->device));
    const int N = env->p.n;
    std::vector<double> tmp((size_t)N * env->E);
    hipStream_t st = as_stream(stream);
    // a packed day mid-day: empty chargers keep the arrival SoC their running SoC carries (sng_layout.h)
    std::vector<uint16_t> rec;
    const bool packed_mid = env->p.packed && env->t >= 1;
    if (packed_mid) {
        rec.resize(tmp.size());
        HIP_TRY(env, hipMemcpyAsync(tmp.data(), env->ds.soc, tmp.size() * sizeof(double), hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipMemcpyAsync(rec.data(), reinterpret_cast<const uint16_t *>(env->ds.aux) + (size_t)env->t * rec.size(),
                                    rec.size() * sizeof(uint16_t), hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipStreamSynchronize(st));
    }
    for (int64_t e = 0; e < env->E; ++e)
        for (int c = 0; c < N; ++c) {
            // the record plane in charger quads, the SoC state in charger pairs (sng_layout.h)
            if (!packed_mid || (rec[rec_index(c, e, N, env->E)] & W_OCC)) tmp[soc_index(c, e, N, env->E)] = h[e * N + c];
        }
    HIP_TRY(env, hipMemcpyAsync(env->ds.soc, tmp.data(), tmp.size() * sizeof(double), hipMemcpyHostToDevice, st));
    HIP_TRY(env, hipStreamSynchronize(st));
    return SNG_OK;
}

// Inverse of encode_day / generate_kernel for envs [first, first + count): the word stream gives
// occupancy, capacity and (at each arrival, W_STATIC on an occupied step) the departure; aux gives the
// arrival SoC and the SOC[c, t] of empty chargers; the req stream holds Requested_SOC[c, t-1] at
// t >= 1 and Requested_SOC[c, T-1] at t = 0.  The env range's columns of each plane come over in one
// 2D copy.
int sng_get_scenario(SngEnv *env, int64_t first, int64_t count, int32_t V, double *soc, double *occupancy,
                     double *capacity, double *requested_soc, int32_t *arrivals, int32_t *departures,
                     int32_t *n_vehicles, double *pv_ratio, void *stream) {
    if (!env || !soc || !occupancy || !capacity || !requested_soc || !arrivals || !departures || !n_vehicles ||
        !pv_ratio)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (first < 0 || count < 1 || first + count > env->E || V < 1)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "env range or max_vehicles out of range");
    if (env->t < 0) return fail(env, SNG_ERR_STATE, "no day yet: call reset()");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    const int N = env->p.n, T = env->p.T, S = env->slots;
    const size_t rows = (size_t)T * N, pitch = (size_t)env->E, cnt = (size_t)count;
    std::vector<uint32_t> w(rows * cnt);
    std::vector<double> aux(rows * cnt), rq;
    std::vector<uint16_t> rec;
    if (env->p.packed) {   // device-RNG day: 2 B packed records in charger quads (sng_layout.h), T + 1 planes
        // rec[plane][c][k] for the env range, one 2D copy (over the planes) per quad row: the range's slots
        // of quad row c0 are one run of count * width records
        rec.resize(rows * cnt + (size_t)N * cnt);
        std::vector<uint16_t> q((size_t)(T + 1) * 4 * cnt);
        for (int c0 = 0; c0 < N; c0 += 4) {
            const int wq = N - c0 < 4 ? N - c0 : 4;
            HIP_TRY(env, hipMemcpy2DAsync(q.data(), cnt * wq * sizeof(uint16_t),
                                          reinterpret_cast<const uint16_t *>(env->ds.aux) + (size_t)c0 * pitch + first * wq,
                                          (size_t)N * pitch * sizeof(uint16_t), cnt * wq * sizeof(uint16_t), (size_t)T + 1,
                                          hipMemcpyDeviceToHost, st));
            HIP_TRY(env, hipStreamSynchronize(st));
            for (int tp = 0; tp <= T; ++tp)
                for (int cc = 0; cc < wq; ++cc)
                    for (size_t k = 0; k < cnt; ++k)
                        rec[((size_t)tp * N + c0 + cc) * cnt + k] = q[(size_t)tp * cnt * wq + k * wq + cc];
        }
    } else {
        HIP_TRY(env, hipMemcpy2DAsync(w.data(), cnt * sizeof(uint32_t), env->ds.word + first, pitch * sizeof(uint32_t),
                                      cnt * sizeof(uint32_t), rows, hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipMemcpy2DAsync(aux.data(), cnt * sizeof(double), env->ds.aux + first, pitch * sizeof(double),
                                      cnt * sizeof(double), rows, hipMemcpyDeviceToHost, st));
    }
    const bool have_req = env->p.req_stream && !env->p.req_zero && env->ds.req;
    if (have_req) {
        rq.resize(rows * cnt);
        HIP_TRY(env, hipMemcpy2DAsync(rq.data(), cnt * sizeof(double), env->ds.req + first, pitch * sizeof(double),
                                      cnt * sizeof(double), rows, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(env, hipMemcpyAsync(pv_ratio, env->ds.ratio + first, cnt * sizeof(double), hipMemcpyDeviceToHost, st));
    HIP_TRY(env, hipStreamSynchronize(st));
    if (env->p.packed) {
        // step t's record is plane t + 1 (as a word: capacity and steps left in the word's fields); an
        // arrival's SoC is carried by the record before it (plane t), and an empty charger shows 0
        const size_t plane = (size_t)N * cnt;
        for (size_t i = 0; i < rows * cnt; ++i) {
            const uint32_t r = rec[plane + i];
            const bool occ = (r & W_OCC) != 0;
            w[i] = occ ? pack_word(true, (r & W_STATIC) != 0, (r & W_PEN) != 0, rec_cap(r), rec_dep(r)) : (r & W_PEN);
            aux[i] = (occ && (r & W_STATIC)) ? (double)rec_soc(rec[i]) : 0.0;
        }
    }
    for (size_t k = 0; k < cnt; ++k) {
        double *soc_k = soc + k * N * S, *occ_k = occupancy + k * N * S, *cap_k = capacity + k * N * S;
        double *req_k = requested_soc + k * N * S;
        int32_t *arr_k = arrivals + k * N * V, *dep_k = departures + k * N * V, *nv_k = n_vehicles + k * N;
        std::fill(soc_k, soc_k + (size_t)N * S, 0.0);
        std::fill(occ_k, occ_k + (size_t)N * S, 0.0);
        std::fill(cap_k, cap_k + (size_t)N * S, 0.0);
        std::fill(req_k, req_k + (size_t)N * S, 0.0);
        std::fill(arr_k, arr_k + (size_t)N * V, -1);
        std::fill(dep_k, dep_k + (size_t)N * V, -1);
        for (int c = 0; c < N; ++c) {
            int nv = 0;
            for (int t = 0; t < T; ++t) {
                const size_t i = ((size_t)t * N + c) * cnt + k;
                const uint32_t word = w[i];
                const bool occ = (word & W_OCC) != 0;
                const size_t o = (size_t)c * S + t;
                if (occ) {
                    occ_k[o] = 1.0;
                    cap_k[o] = (double)((word >> W_CAP_SHIFT) & 0xffu);
                    if (word & W_STATIC) {   // arrival: SOC[c, t] as generated, departure t + remaining
                        soc_k[o] = aux[i];
                        if (nv < V) {
                            arr_k[(size_t)c * V + nv] = t;
                            dep_k[(size_t)c * V + nv] = t + (int)((word >> W_DEP_SHIFT) & 0xffu);
                        }
                        ++nv;
                    }
                } else {
                    soc_k[o] = aux[i];
                }
                if (have_req)
                    req_k[o] = rq[((t + 1 < T ? (size_t)(t + 1) * N : 0) + c) * cnt + k];
                else   // a replayed day keeps the cleared zeros (charging_station.py:138-150)
                    req_k[o] = (occ && !env->p.req_zero) ? 1.0 : 0.0;
            }
            nv_k[c] = nv;
        }
    }
    return SNG_OK;
}

int sng_get_tables(const SngEnv *env, double *irr, double *irr_max, double *pv_power, double *price,
                   double *price_max, int32_t *n) {
    if (!env) return SNG_ERR_INVALID_ARGUMENT;
    const auto &tb = env->tables;
    if (irr) std::memcpy(irr, tb.irr.data(), tb.irr.size() * sizeof(double));
    if (pv_power) std::memcpy(pv_power, tb.pv_power.data(), tb.pv_power.size() * sizeof(double));
    if (price) std::memcpy(price, tb.price.data(), tb.price.size() * sizeof(double));
    if (irr_max) *irr_max = tb.irr_max;
    if (price_max) *price_max = tb.price_max;
    if (n) *n = (int32_t)tb.irr.size();
    return SNG_OK;
}

// ---------------------------------------------------------------------------------
// Checkpoint / resume: header, then the sections in this order (host byte order):
//   soc f64[N/2][E][2] (charger pairs) | bess, bess0, ratio, pen0 f64[E] | flags u32[E] | [word u32[T][N][E], host days]
//   | aux 8B[T][N][E] (a packed day: its u16 records in charger quads, sng_layout.h) | [req f64[T][N][E]]
//   | [profile keys u32[E][2]] | [episode return f64[E]]
//   | [reference streams u32[E][2][625]]
// ---------------------------------------------------------------------------------
struct StateHeader {
    char magic[8];
    int32_t abi, header_bytes;
    int64_t num_envs;
    int32_t n, T, slots, obs_dim;
    uint64_t config_hash, seed;
    int64_t env_offset;
    int32_t t, day_finished;
    int32_t packed, req_stream, req_zero, bump_day;
    int32_t gen_mode, gen_loaded;
    uint64_t replays, day_counter;
    int32_t has_word, has_req, has_prof, has_return, has_streams, reserved;
    uint64_t total_bytes;
};
// the last byte is the checkpoint format version: '3' since the configuration fingerprint is hashed
// field by field (round 3), '5' since the SoC state is stored in charger pairs, a day's stochastic profiles
// as per-env keys and a device day's records in 2 B (round 4); a blob of another version is refused as such
static const char kStateMagic[8] = {'S', 'N', 'G', 'S', 'T', 'A', 'T', '5'};

// The blob's size for this handle and the header's section flags.
static uint64_t state_bytes(const SngEnv *env, const StateHeader &h) {
    const size_t E = (size_t)env->E, tl = env->timeline();
    size_t b = sizeof(StateHeader) + (size_t)env->p.n * E * 8 + 4 * E * 8 + E * 4 + tl * 8;
    if (h.has_word) b += tl * 4;
    if (h.has_req) b += tl * 8;
    if (h.has_prof) b += 2 * (size_t)E * 4;
    if (h.has_return) b += E * 8;
    if (h.has_streams) b += E * 2 * MT19937::kStateWords * 4;
    return b;
}

static StateHeader state_layout(const SngEnv *env, bool with_return) {
    StateHeader h{};
    std::memcpy(h.magic, kStateMagic, sizeof h.magic);
    h.abi = SNG_ABI_VERSION;
    h.header_bytes = (int32_t)sizeof(StateHeader);
    h.num_envs = env->E;
    h.n = env->p.n;
    h.T = env->p.T;
    h.slots = env->slots;
    h.obs_dim = env->p.obs_dim;
    h.config_hash = env->cfg_hash;
    h.seed = env->seed;
    h.env_offset = env->p.env_offset;
    h.t = env->t;
    h.day_finished = env->day_finished ? 1 : 0;
    h.packed = env->p.packed;
    h.req_stream = env->p.req_stream;
    h.req_zero = env->p.req_zero;
    h.bump_day = env->p.bump_day;
    h.gen_mode = env->gen_mode;
    h.gen_loaded = env->gen_loaded ? 1 : 0;
    h.replays = env->replays;
    h.has_word = env->p.packed ? 0 : 1;
    h.has_req = (env->ds.req && env->p.req_stream) ? 1 : 0;
    h.has_prof = env->ds.prof_key ? 1 : 0;
    h.has_return = with_return ? 1 : 0;
    h.has_streams = env->py_seeded ? 1 : 0;
    h.total_bytes = state_bytes(env, h);
    return h;
}

int sng_state_size(const SngEnv *env, int with_return, size_t *bytes) {
    if (!env || !bytes) return SNG_ERR_INVALID_ARGUMENT;
    *bytes = (size_t)state_layout(env, with_return != 0).total_bytes;
    return SNG_OK;
}

int sng_get_state(SngEnv *env, void *buf, size_t bytes, const double *episode_return, void *stream) {
    if (!env || !buf) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    StateHeader h = state_layout(env, episode_return != nullptr);
    if (bytes < h.total_bytes) return fail(env, SNG_ERR_INVALID_ARGUMENT, "state buffer too small (sng_state_size)");
    const size_t E = (size_t)env->E, tl = env->timeline();
    char *out = static_cast<char *>(buf) + sizeof(StateHeader);
    auto pull = [&](const void *dev, size_t n) -> hipError_t {
        hipError_t e = hipMemcpyAsync(out, dev, n, hipMemcpyDeviceToHost, st);
        out += n;
        return e;
    };
    // the numpy streams live on the device: seeded here if no reference day drew from them yet
    std::vector<uint32_t> np_words, py_words;
    std::vector<int32_t> np_pos, py_pos;
    if (h.has_streams) {
        int rc = ensure_np_streams(env, st);
        if (rc) return rc;
        rc = await_prepare(env, st);
        if (rc) return rc;
        np_words.resize(E * 2 * kMtN);
        py_words.resize(E * 2 * kMtN);
        np_pos.resize(E);
        py_pos.resize(E);
        HIP_TRY(env, hipMemcpyAsync(np_words.data(), env->rs.mt, np_words.size() * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipMemcpyAsync(np_pos.data(), env->rs.pos, E * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipMemcpyAsync(py_words.data(), env->ps.mt, py_words.size() * 4, hipMemcpyDeviceToHost, st));
        HIP_TRY(env, hipMemcpyAsync(py_pos.data(), env->ps.pos, E * 4, hipMemcpyDeviceToHost, st));
    }
    HIP_TRY(env, hipMemcpyAsync(&h.day_counter, env->ds.episode, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(env, pull(env->ds.soc, (size_t)env->p.n * E * 8));
    HIP_TRY(env, pull(env->ds.bess, E * 8));
    HIP_TRY(env, pull(env->ds.bess0, E * 8));
    HIP_TRY(env, pull(env->ds.ratio, E * 8));
    HIP_TRY(env, pull(env->ds.pen0, E * 8));
    HIP_TRY(env, pull(env->ds.flags, E * 4));
    if (h.has_word) HIP_TRY(env, pull(env->ds.word, tl * 4));
    HIP_TRY(env, pull(env->ds.aux, tl * 8));
    if (h.has_req) HIP_TRY(env, pull(env->ds.req, tl * 8));
    if (h.has_prof) HIP_TRY(env, pull(env->ds.prof_key, 2 * (size_t)E * 4));
    if (h.has_return) HIP_TRY(env, pull(episode_return, E * 8));
    HIP_TRY(env, hipStreamSynchronize(st));
    if (h.has_streams) {
        uint32_t *w = reinterpret_cast<uint32_t *>(out);
        for (size_t i = 0; i < E; ++i) {
            // numpy's RandomState, then Python's random: each the current block's 624 words and mti
            // (the layout of sng_mt.h MT19937::save)
            for (int k = 0; k < 2; ++k) {
                const std::vector<uint32_t> &words = k ? py_words : np_words;
                const int32_t pos = k ? py_pos[i] : np_pos[i];
                uint32_t *o = w + (2 * i + k) * MT19937::kStateWords;
                const int cur = (pos >> 16) & 1, mti = pos & kMtPosMask;
                const uint32_t *src = words.data() + (i * 2 + cur) * kMtN;
                for (int k = 0; k < kMtN; ++k) o[k] = mt_untemper_word(src[k]);   // the raw state
                o[kMtN] = (uint32_t)mti;
            }
        }
    }
    std::memcpy(buf, &h, sizeof h);
    return SNG_OK;
}

int sng_set_state(SngEnv *env, const void *buf, size_t bytes, double *episode_return, void *stream) {
    if (!env || !buf) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (bytes < sizeof(StateHeader)) return fail(env, SNG_ERR_INVALID_ARGUMENT, "not an sng state");
    StateHeader h;
    std::memcpy(&h, buf, sizeof h);
    if (std::memcmp(h.magic, kStateMagic, sizeof h.magic - 1) == 0 && h.magic[7] != kStateMagic[7])
        return fail(env, SNG_ERR_INVALID_ARGUMENT,
                    std::string("unsupported checkpoint version ") + h.magic[7] + " (this library reads version " +
                        kStateMagic[7] + ")");
    if (std::memcmp(h.magic, kStateMagic, sizeof h.magic) != 0 || h.abi != SNG_ABI_VERSION ||
        h.header_bytes != (int32_t)sizeof(StateHeader))
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "not an sng state of this ABI version");
    if (h.num_envs != env->E || h.n != env->p.n || h.T != env->p.T || h.slots != env->slots ||
        h.obs_dim != env->p.obs_dim || h.config_hash != env->cfg_hash)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "state of a handle with another configuration or size");
    // the sections the header announces must be self-consistent before any of them is read
    auto flag = [](int32_t v) { return v == 0 || v == 1; };
    if (!flag(h.has_word) || !flag(h.has_req) || !flag(h.has_prof) || !flag(h.has_return) || !flag(h.has_streams) ||
        !flag(h.packed) || h.has_word != 1 - h.packed || state_bytes(env, h) != h.total_bytes)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "corrupt state header (inconsistent sections or size)");
    if (h.total_bytes > bytes) return fail(env, SNG_ERR_INVALID_ARGUMENT, "truncated state");
    if (h.has_return && !episode_return)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "the state holds day returns: pass an episode_return array");
    if ((h.has_prof != 0) != (env->ds.prof_key != nullptr)) return fail(env, SNG_ERR_INVALID_ARGUMENT, "profile mismatch");
    if (h.t < -1 || h.t > env->p.T) return fail(env, SNG_ERR_INVALID_ARGUMENT, "bad timestep in state");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    if (h.has_req) {
        int rc = ensure_req(env);
        if (rc) return rc;
    }
    const size_t E = (size_t)env->E, tl = env->timeline();
    const char *in = static_cast<const char *>(buf) + sizeof(StateHeader);
    auto push = [&](void *dev, size_t n) -> hipError_t {
        hipError_t e = hipMemcpyAsync(dev, in, n, hipMemcpyHostToDevice, st);
        in += n;
        return e;
    };
    // the restored streams, checked before anything is changed: Python's into host streams, numpy's
    // into block 0 of the device streams (position = mti)
    std::vector<uint32_t> np_words, py_words;
    std::vector<int32_t> np_pos, py_pos;
    if (h.has_streams) {
        const size_t off = h.total_bytes - E * 2 * MT19937::kStateWords * 4;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(static_cast<const char *>(buf) + off);
        np_words.resize(E * kMtN);
        py_words.resize(E * kMtN);
        np_pos.resize(E);
        py_pos.resize(E);
        for (size_t i = 0; i < E; ++i) {
            for (int k = 0; k < 2; ++k) {
                const uint32_t *src = w + (2 * i + k) * MT19937::kStateWords;
                if (src[kMtN] > (uint32_t)kMtN + 1)
                    return fail(env, SNG_ERR_INVALID_ARGUMENT, "corrupt RNG stream state");
                uint32_t *dst = (k ? py_words : np_words).data() + i * kMtN;
                for (int q = 0; q < kMtN; ++q) dst[q] = mt_temper_word(src[q]);   // RefStreams keep tempered words
                // mti = N + 1 (never seeded) cannot come from a seeded generator
                (k ? py_pos : np_pos)[i] = (int32_t)std::min<uint32_t>(src[kMtN], (uint32_t)kMtN);
            }
        }
        for (RefStreams *r : {&env->rs, &env->ps}) {
            if (!r->mt) {
                HIP_TRY(env, hipMalloc(&r->mt, E * 2 * kMtN * sizeof(uint32_t)));
                HIP_TRY(env, hipMalloc(&r->pos, E * sizeof(int32_t)));
            }
        }
        int rc = await_prepare(env, st);   // no preparation may still be writing the streams
        if (rc) return rc;
    }
    HIP_TRY(env, hipMemcpyAsync(env->ds.episode, &h.day_counter, sizeof(uint64_t), hipMemcpyHostToDevice, st));
    HIP_TRY(env, push(env->ds.soc, (size_t)env->p.n * E * 8));
    HIP_TRY(env, push(env->ds.bess, E * 8));
    HIP_TRY(env, push(env->ds.bess0, E * 8));
    HIP_TRY(env, push(env->ds.ratio, E * 8));
    HIP_TRY(env, push(env->ds.pen0, E * 8));
    HIP_TRY(env, push(env->ds.flags, E * 4));
    if (h.has_word) HIP_TRY(env, push(env->ds.word, tl * 4));
    HIP_TRY(env, push(env->ds.aux, tl * 8));
    if (h.has_req) HIP_TRY(env, push(env->ds.req, tl * 8));
    if (h.has_prof) HIP_TRY(env, push(env->ds.prof_key, 2 * (size_t)E * 4));
    if (h.has_return) HIP_TRY(env, push(episode_return, E * 8));
    if (h.has_streams) {
        HIP_TRY(env, hipMemcpy2DAsync(env->rs.mt, 2 * kMtN * sizeof(uint32_t), np_words.data(), kMtN * sizeof(uint32_t),
                                      kMtN * sizeof(uint32_t), E, hipMemcpyHostToDevice, st));
        HIP_TRY(env, hipMemcpyAsync(env->rs.pos, np_pos.data(), E * sizeof(int32_t), hipMemcpyHostToDevice, st));
        HIP_TRY(env, hipMemcpy2DAsync(env->ps.mt, 2 * kMtN * sizeof(uint32_t), py_words.data(), kMtN * sizeof(uint32_t),
                                      kMtN * sizeof(uint32_t), E, hipMemcpyHostToDevice, st));
        HIP_TRY(env, hipMemcpyAsync(env->ps.pos, py_pos.data(), E * sizeof(int32_t), hipMemcpyHostToDevice, st));
    }
    HIP_TRY(env, hipStreamSynchronize(st));
    env->seed = h.seed;
    env->p.seed = h.seed;
    env->p.env_offset = h.env_offset;
    env->t = h.t;
    env->day_finished = h.day_finished != 0;
    env->p.packed = h.packed;
    env->p.req_stream = h.req_stream;
    env->p.req_zero = h.req_zero;
    env->p.bump_day = h.bump_day;
    env->gen_mode = h.gen_mode;
    env->gen_loaded = h.gen_loaded != 0;
    env->replays = h.replays;
    env->np_seeded = h.has_streams != 0;
    env->py_seeded = h.has_streams != 0;
    env->prepared = false;   // the restored position says what the next day still has to prepare
    return SNG_OK;
}

int sng_graph_create(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done,
                     const SngInfo *info, int flags, int32_t days, double *day_returns, SngGraph **out) {
    const bool with_reset = (flags & SNG_GRAPH_RESET) != 0;
    if (!env || !actions || !obs || !reward || !done || !out) return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (days < 1 || (days > 1 && !with_reset))
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "days must be >= 1 (more than one needs SNG_GRAPH_RESET)");
    if (with_reset && !device_rng_ok(env))
        return fail(env, SNG_ERR_UNSUPPORTED, "device RNG needs time_interval <= 2h");
    HIP_TRY(env, hipSetDevice(env->device));
    if (env->p.req_enabled) {
        int rc = ensure_req(env);
        if (rc) return rc;
    }
    hipStream_t cs;
    HIP_TRY(env, hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    SngGraph *g = new SngGraph();
    g->env = env;
    Params p = env->p;
    if (with_reset) {   // every day a freshly generated device day (sng_reset(SNG_RNG_DEVICE))
        p.req_stream = p.req_enabled;
        p.packed = 1;
        p.req_zero = 0;
        p.bump_day = 1;
    }
    g->with_reset = with_reset;
    g->key = day_key(p);
    g->seed = env->seed;
    g->env_offset = p.env_offset;
    const InfoPtrs ip = info_ptrs(info);
    const int64_t E = env->E;
    const int A = p.act_dim;
    const int vec = (aligned16(actions) && aligned16(obs)) ? 1 : 0;
    hipError_t e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    for (int d = 0; e == hipSuccess && d < days; ++d) {
        InfoPtrs ipd = ip;   // day d's returns into row d (observe0 zeroes it, every step adds)
        if (day_returns) ipd.episode_return = day_returns + (size_t)d * E;
        if (with_reset) {
            e = launch_generate(p, env->ds, env->seed, E, env->i4, env->i10, env->i1, obs, ipd.episode_return, vec, cs);
        }
        for (int t = 0; e == hipSuccess && t < p.T; ++t)
            e = launch_step(p, env->ds, ipd, env->host_tab, actions + (size_t)t * E * A, obs, reward, done, E, t, vec, cs);
    }
    hipGraph_t graph = nullptr;
    hipError_t e2 = hipStreamEndCapture(cs, &graph);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) e = hipGraphInstantiate(&g->exec, graph, nullptr, nullptr, 0);
    (void)hipStreamDestroy(cs);
    if (e != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        delete g;
        return hip_fail(env, e, "graph capture");
    }
    g->graph = graph;
    *out = g;
    return SNG_OK;
}

int sng_graph_launch(SngGraph *g, void *stream) {
    if (!g) return SNG_ERR_INVALID_ARGUMENT;
    SngEnv *env = g->env;
    if (!g->with_reset) {
        // a steps-only graph steps the loaded day from t = 0 with the Params it was captured with
        if (!(g->key == day_key(env->p)))
            return fail(env, SNG_ERR_STATE,
                        "graph captured for a day of another encoding (RNG mode, requested-SoC stream or replay): "
                        "recapture it after this reset");
        if (env->t != 0) return fail(env, SNG_ERR_STATE, "a steps-only graph starts at t = 0: reset first");
    }
    // sng_set_seed / sng_set_state / sng_set_env_offset since the capture: the graph's kernels would
    // still draw the old streams
    if (g->seed != env->seed || g->env_offset != env->p.env_offset)
        return fail(env, SNG_ERR_STATE, "seed or env offset changed since the graph was captured: recapture it");
    HIP_TRY(env, hipSetDevice(env->device));
    // the graph's first reset must not redraw a device day that was reset but never stepped
    if (g->with_reset && env->p.packed && env->p.bump_day && env->t == 0)
        HIP_TRY(env, launch_bump_day(env->ds, as_stream(stream)));
    HIP_TRY(env, hipGraphLaunch(g->exec, as_stream(stream)));
    if (g->with_reset) {
        env->p.req_stream = env->p.req_enabled;
        env->p.packed = 1;
        env->p.req_zero = 0;
        env->p.bump_day = 1;
        env->gen_mode = SNG_RNG_DEVICE;
        env->gen_loaded = true;
    }
    env->t = env->p.T;
    env->day_finished = true;
    return SNG_OK;
}

void sng_graph_destroy(SngGraph *g) {
    if (!g) return;
    (void)hipSetDevice(g->env->device);
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->graph) (void)hipGraphDestroy(g->graph);
    delete g;
}

int sng_time_step_kernels(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done,
                          const SngInfo *info, int32_t days, float *ms, float *reset_ms, void *stream) {
    if (!env || !actions || !obs || !reward || !done || days < 1)
        return fail(env, SNG_ERR_INVALID_ARGUMENT, "null argument");
    if (!device_rng_ok(env)) return fail(env, SNG_ERR_UNSUPPORTED, "device RNG needs time_interval <= 2h");
    HIP_TRY(env, hipSetDevice(env->device));
    hipStream_t st = as_stream(stream);
    Params p = env->p;
    p.req_stream = p.req_enabled;
    p.packed = 1;
    p.req_zero = 0;
    p.bump_day = 1;
    if (p.req_stream) {
        int rc = ensure_req(env);
        if (rc) return rc;
    }
    const InfoPtrs ip = info_ptrs(info);
    const int64_t E = env->E;
    const int T = p.T, A = p.act_dim;
    const int vec = (aligned16(actions) && aligned16(obs)) ? 1 : 0;
    std::vector<hipEvent_t> ev(ms ? 2 * (size_t)T * days : 0, nullptr), rev(reset_ms ? 2 * (size_t)days : 0, nullptr);
    hipError_t e = hipSuccess;
    if (env->p.packed && env->p.bump_day && env->t == 0) e = launch_bump_day(env->ds, st);   // as in sng_reset
    for (auto &x : ev)
        if (e == hipSuccess) e = hipEventCreate(&x);
    for (auto &x : rev)
        if (e == hipSuccess) e = hipEventCreate(&x);
    for (int d = 0; e == hipSuccess && d < days; ++d) {
        e = launch_generate(p, env->ds, env->seed, E, env->i4, env->i10, env->i1, obs, ip.episode_return, vec, st,
                            reset_ms ? rev[2 * (size_t)d] : nullptr, reset_ms ? rev[2 * (size_t)d + 1] : nullptr);
        for (int t = 0; e == hipSuccess && t < T; ++t) {
            hipEvent_t a = ms ? ev[2 * ((size_t)d * T + t)] : nullptr, b = ms ? ev[2 * ((size_t)d * T + t) + 1] : nullptr;
            e = launch_step(p, env->ds, ip, env->host_tab, actions + (size_t)t * E * A, obs, reward, done, E, t, vec, st, a, b);
        }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    for (int k = 0; e == hipSuccess && ms && k < T * days; ++k) e = hipEventElapsedTime(&ms[k], ev[2 * k], ev[2 * k + 1]);
    for (int d = 0; e == hipSuccess && reset_ms && d < days; ++d)
        e = hipEventElapsedTime(&reset_ms[d], rev[2 * (size_t)d], rev[2 * (size_t)d + 1]);
    for (auto x : ev)
        if (x) (void)hipEventDestroy(x);
    for (auto x : rev)
        if (x) (void)hipEventDestroy(x);
    if (e != hipSuccess) return hip_fail(env, e, "timed day");
    env->p.req_stream = p.req_stream;
    env->p.packed = 1;
    env->p.req_zero = 0;
    env->p.bump_day = 1;
    env->gen_mode = SNG_RNG_DEVICE;
    env->gen_loaded = true;
    env->t = T;
    env->day_finished = true;
    return SNG_OK;
}

int sng_bandwidth_probe(int device, int64_t read_bytes, int64_t write_bytes, int32_t reps, float *dispatch_us,
                        float *back_to_back_us, void *stream) {
    if (read_bytes < 0 || write_bytes < 0 || read_bytes + write_bytes < 16 || reps < 1)
        return fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "sng_bandwidth_probe: bad sizes");
    if (hipSetDevice(device) != hipSuccess) return fail(nullptr, SNG_ERR_HIP, "sng_bandwidth_probe: hipSetDevice");
    hipStream_t st = as_stream(stream);
    const int64_t nr = read_bytes / 16, nw = write_bytes / 16;
    void *in = nullptr, *out = nullptr;
    std::vector<hipEvent_t> ev(2 * (size_t)reps + 2, nullptr);
    hipError_t e = hipMalloc(&in, (size_t)std::max<int64_t>(nr, 1) * 16);
    if (e == hipSuccess) e = hipMalloc(&out, (size_t)std::max<int64_t>(nw, 1) * 16);
    if (e == hipSuccess) e = hipMemsetAsync(in, 0, (size_t)std::max<int64_t>(nr, 1) * 16, st);
    for (auto &x : ev)
        if (e == hipSuccess) e = hipEventCreate(&x);
    // warm-up, then `reps` dispatches each between its own start/stop events (the dispatch's device time),
    // then `reps` back to back between two events (start to start, as a graph runs kernels)
    for (int k = 0; e == hipSuccess && k < 3; ++k) e = launch_probe_copy(in, out, nr, nw, st, nullptr, nullptr);
    for (int k = 0; e == hipSuccess && k < reps; ++k)
        e = launch_probe_copy(in, out, nr, nw, st, ev[2 * (size_t)k], ev[2 * (size_t)k + 1]);
    if (e == hipSuccess) e = hipEventRecord(ev[2 * (size_t)reps], st);
    for (int k = 0; e == hipSuccess && k < reps; ++k) e = launch_probe_copy(in, out, nr, nw, st, nullptr, nullptr);
    if (e == hipSuccess) e = hipEventRecord(ev[2 * (size_t)reps + 1], st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    float sum = 0.f, ms = 0.f;
    for (int k = 0; e == hipSuccess && k < reps; ++k) {
        e = hipEventElapsedTime(&ms, ev[2 * (size_t)k], ev[2 * (size_t)k + 1]);
        sum += ms;
    }
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, ev[2 * (size_t)reps], ev[2 * (size_t)reps + 1]);
    for (auto x : ev)
        if (x) (void)hipEventDestroy(x);
    if (in) (void)hipFree(in);
    if (out) (void)hipFree(out);
    if (e != hipSuccess) return fail(nullptr, SNG_ERR_HIP, std::string("sng_bandwidth_probe: ") + hipGetErrorString(e));
    if (dispatch_us) *dispatch_us = sum / reps * 1e3f;
    if (back_to_back_us) *back_to_back_us = ms / reps * 1e3f;
    return SNG_OK;
}

int sng_host_generate_scenarios(const SngConfig *cfg, int64_t num_envs, uint64_t seed, int32_t episodes, double *soc,
                                double *occupancy, double *capacity, double *requested_soc, int32_t *arrivals,
                                int32_t *departures, int32_t max_vehicles, double *pv_ratio) {
    int T = 0;
    std::string err;
    int rc = validate(cfg, &T, err);
    if (rc) return fail(nullptr, rc, err);
    if (num_envs < 1 || episodes < 1 || max_vehicles < 1)
        return fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "bad sizes");
    const int N = cfg->number_of_chargers;
    const int S = cfg->extended_day ? T + 1 : kSlots;
    bool overflow = false;
    for (int64_t i = 0; i < num_envs; ++i) {
        MT19937 np_rng, py_rng;
        np_rng.seed_numpy((uint32_t)(seed + (uint64_t)i));
        py_rng.seed_python(seed + (uint64_t)i);
        for (int ep = 0; ep < episodes; ++ep) {
            if (ep > 0) (void)py_rng.py_randint(0, 180);   // day-end draw, smart_nanogrid_environment.py:181
            const size_t k = (size_t)ep * num_envs + i;
            DayView d{soc + k * N * S, occupancy + k * N * S, capacity + k * N * S, requested_soc + k * N * S,
                      arrivals + k * N * max_vehicles, departures + k * N * max_vehicles, max_vehicles, S};
            if (!generate_day(*cfg, T, np_rng, d)) overflow = true;
            pv_ratio[k] = (double)py_rng.py_randint(0, 180) / 100;
        }
    }
    if (overflow) return fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "max_vehicles too small");
    return SNG_OK;
}

int32_t sng_host_threads(void) { return host_threads(); }

int sng_get_day_counter(SngEnv *env, uint64_t *out, void *stream) {
    if (!env) return SNG_ERR_INVALID_ARGUMENT;
    if (!out) return fail(env, SNG_ERR_INVALID_ARGUMENT, "sng_get_day_counter: null output");
    HIP_TRY(env, hipSetDevice(env->device));
    HIP_TRY(env, hipMemcpyAsync(out, env->ds.episode, sizeof(uint64_t), hipMemcpyDeviceToHost, as_stream(stream)));
    HIP_TRY(env, hipStreamSynchronize(as_stream(stream)));
    return SNG_OK;
}

}  // extern "C"
