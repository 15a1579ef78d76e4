/*
 * sng.h -- C ABI of the MI355X-native batched SmartNanogridEnv (libsng.so).
 *
 * Drop-in boundary for the reference's step()/reset() hot path.  The reference
 * (Dellintel98/smart-nanogrid-gym, pure Python) has no FFI of its own; its
 * plugin surface is the gym.Env it registers as 'SmartNanogridEnv-v0'
 * (smart_nanogrid_gym/__init__.py:4-8).  Each entry point below names the
 * reference interface it replaces.  The Python mirror of that interface
 * (smart-nanogrid-gym_amd/smart_nanogrid_gym/) binds these symbols with ctypes;
 * INTEGRATION.md shows the binding.
 *
 * Conventions
 *   - Plain C types only.  Device buffers are raw device pointers (e.g. a torch
 *     tensor's data_ptr()); `stream` is an opaque hipStream_t (NULL = default).
 *   - Every call returns SNG_OK (0) or a negative SngStatus; the message is in
 *     sng_last_error(env) (or sng_last_error(NULL) for sng_create failures).
 *   - All calls on one handle must come from one host thread at a time.
 *   - Layouts at the boundary: actions float32 [num_envs][act_dim] row-major,
 *     observations float32 [num_envs][obs_dim] row-major, reward float64
 *     [num_envs], done uint8 [num_envs] -- exactly the per-env arrays the
 *     reference returns, stacked.
 */
#ifndef SNG_H
#define SNG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNG_ABI_VERSION 10

typedef enum SngStatus {
    SNG_OK = 0,
    SNG_ERR_INVALID_ARGUMENT = -1,   /* ValueError in the reference */
    SNG_ERR_UNSUPPORTED = -2,        /* configuration the reference cannot run either */
    SNG_ERR_HIP = -3,                /* HIP runtime failure */
    SNG_ERR_STATE = -4,              /* call out of order (e.g. step before reset) */
    SNG_ERR_OUT_OF_MEMORY = -5
} SngStatus;

/* vehicle_uncharged_penalty_mode, charging_station.py:50-60 */
typedef enum SngPenaltyMode {
    SNG_PENALTY_NONE = 0,            /* 'no_penalty' */
    SNG_PENALTY_ON_DEPARTURE = 1,    /* 'on_departure' */
    SNG_PENALTY_SPARSE = 2,          /* 'sparse' */
    SNG_PENALTY_DENSE = 3            /* 'dense' */
} SngPenaltyMode;

/* How sng_reset draws the new day's vehicles. */
typedef enum SngRngMode {
    /* Host MT19937 streams identical to the reference's global RNGs: environment i
     * reproduces `np.random.seed(seed + i); random.seed(seed + i)` followed by the
     * reference's reset()/step() sequence (charging_station.py:200-279,
     * smart_nanogrid_environment.py:181,349).  Generated on the host CPU threads. */
    SNG_RNG_REFERENCE = 0,
    /* Counter-based hash streams on the GPU: same distributions, different draws (the arrival
     * SoC is drawn as a float32 value).  Fully device-resident; graph-capturable.  Each device
     * reset draws a new day of the handle's day counter, which the day's first step advances. */
    SNG_RNG_DEVICE = 1
} SngRngMode;

/* Per-env flag bits reported by sng_read_errors / SngInfo.flags. */
#define SNG_FLAG_SUMMARY_WORDS 1024   /* SngInfo.flag_summary's words */
#define SNG_FLAG_NEGATIVE_DEMAND  0x1u  /* ValueError, central_management_system.py:158-159 */
#define SNG_FLAG_CHARGING_MODE    0x2u  /* ValueError, charger.py:88/138, battery_energy_storage_system.py:74/106 */
#define SNG_FLAG_BESS_SOC_ABOVE_1 0x4u  /* ValueError, penaliser.py:110-111 */
#define SNG_FLAG_V2X_BREAKPOINT   0x8u  /* breakpoint(), central_management_system.py:160-165 (not an error) */

/* Constructor keyword arguments of SmartNanogridEnv (smart_nanogrid_environment.py:32-34)
 * plus the module constants the reference hard-codes, with the reference's values as
 * defaults (sng_config_defaults). */
typedef struct SngConfig {
    int32_t abi_version;                     /* = SNG_ABI_VERSION */
    int32_t number_of_chargers;              /* N (1..128) */
    double time_interval_hours;              /* set_time_interval(), :125-138 ('1h' -> 1.0) */
    int32_t price_model;                     /* accountant.py:58-101, 0..4 */
    int32_t pv_system_available;             /* pv_system_available_in_model */
    int32_t battery_system_available;        /* battery_system_available_in_model */
    int32_t vehicle_to_everything;           /* vehicle_to_everything */
    int32_t different_vehicle_capacities;    /* enable_different_vehicle_battery_capacities */
    int32_t requested_state_of_charge;       /* enable_requested_state_of_charge */
    int32_t charging_mode_bounded;           /* charging_mode == 'bounded' */
    int32_t penalty_mode;                    /* SngPenaltyMode */
    int32_t numpy_legacy_promotion;          /* 1: NumPy<2 float64 EV power (the recorded KATs) */
    double grid_cost_weight;                 /* accountant.py:35 -> 0.75 */
    double battery_penalty_weight;           /* penaliser.py:181 -> 0.8 */
    double selling_price_coefficient;        /* accountant.py:6 -> 0.8 */
    /* BESS, central_management_system.py:35 */
    double bess_capacity_kwh;                /* 80 */
    double bess_initial_soc;                 /* 0.5 */
    double bess_max_charging_kw;             /* 44 */
    double bess_max_discharging_kw;          /* 44 */
    double bess_charging_efficiency;         /* 0.95 */
    double bess_discharging_efficiency;      /* 0.95 */
    double bess_depth_of_discharge;          /* 0.15 */
    /* EV charger, charger.py:20-23 */
    double ev_max_power_kw;                  /* 22 */
    double ev_efficiency;                    /* 0.95 */
    /* PV input: per-minute irradiance (W/m^2), solar_irradiance.mat['irradiance'] */
    const double *irradiance_per_minute;
    int64_t irradiance_minutes;
    /* Kernel tuning: GPU lanes per environment in the step kernel (0 = automatic; 1, 2, 4). */
    int32_t step_lanes_per_env;
    /* Build-defined generalisation (no reference oracle, default off):
     * extended_day = 1 allows days longer than 24 steps (dt < 1 h): per-charger arrays get
     * T+1 slots, prices come from the per-step tariff loop (accountant.py:61-68).
     * pv_noise / price_noise = sigma > 0 scale every PV / price table entry an env uses on a day
     * by 1 + sigma*z, z in [-1, 1) from a counter-based hash of (env seed, day, k). */
    int32_t extended_day;
    int32_t reserved0;
    double pv_noise;
    double price_noise;
} SngConfig;

typedef struct SngDims {
    int32_t obs_dim;        /* smart_nanogrid_environment.py:90-96 */
    int32_t act_dim;        /* :101-118 */
    int32_t timesteps;      /* 24 / dt */
    int32_t number_of_chargers;
    int64_t num_envs;
    int32_t step_lanes_per_env;   /* lanes per env the step kernel runs with (SngConfig 0 = default) */
    int32_t slots;                /* per-charger scenario array length: 25, or T+1 with extended_day */
} SngDims;

/* Optional per-step diagnostics: device pointers, each [num_envs]; NULL = not written.
 * Names follow the results dict of CentralManagementSystem.manage_nanogrid
 * (central_management_system.py:128-155). */
typedef struct SngInfo {
    double *grid_power;                  /* 'Grid power' */
    double *total_charging_power;        /* 'Total charging power' */
    double *total_discharging_power;     /* 'Total discharging power' */
    double *battery_state_of_charge;     /* 'Battery state of charge' */
    double *total_vehicle_penalty;       /* 'Total vehicle penalty' */
    double *total_battery_penalty;       /* 'Total battery penalty' */
    double *grid_energy_cost;            /* 'Grid energy cost' */
    double *total_cost;                  /* 'Total cost' */
    double *utilized_solar_energy;       /* 'Utilized solar energy' */
    double *battery_power_value;         /* 'Battery power value' */
    double *battery_calculated_power;    /* 'Battery calculated power value' */
    double *nonexistent_vehicle_penalty; /* 'DisCharging nonexistent vehicles penalty' */
    double *initial_battery_soc;         /* 'Initial battery state of charge' */
    uint32_t *flags;                     /* SNG_FLAG_* raised by this step */
    double *episode_return;              /* accumulated: += reward (zeroed by every reset) */
    /* per charger, [num_envs][N] (row-major, env-major); NULL = not written */
    double *charger_power;               /* 'Charger power values' (charging_station.py:282-299) */
    double *vehicle_soc;                 /* SOC[c, t] after the step (charger.py:37-56/:86/:136) */
    /* device u32 [SNG_FLAG_SUMMARY_WORDS], NULL = not written: OR of the SNG_FLAG_* any env raised since the
     * caller last zeroed it, spread over SNG_FLAG_SUMMARY_WORDS words (the envs of one wavefront share a
     * word: word (first env of the wavefront / 32) mod SNG_FLAG_SUMMARY_WORDS), touched only when a flag is
     * raised, one atomic per wavefront.  A caller that watches these words instead of `flags` spares the step
     * its per-env flag store, and reads which envs raised what with sng_read_errors(clear = 1) only when a
     * word is non-zero.  (One shared word made every flagged wavefront's atomic wait on the same address: a
     * V2X station, which flags most envs every step, took ~10 us more per step at 65,536 envs.) */
    uint32_t *flag_summary;
} SngInfo;

/* A scenario in the reference's own layout (ChargingStation after
 * generate_new_initial_values / load_initial_values, charging_station.py:119-186):
 * per env and charger, 25-slot arrays plus padded arrival/departure lists (-1 = none). */
typedef struct SngScenario {
    int32_t slots;                 /* 25 (charger.py:16-19); T+1 with extended_day */
    int32_t max_vehicles;          /* padded list length */
    const double *soc;             /* [num_envs][N][slots]  'SOC' */
    const double *occupancy;       /* [num_envs][N][slots]  'Charger_occupancy' */
    const double *capacity;        /* [num_envs][N][slots]  'Vehicle_capacities' */
    const double *requested_soc;   /* [num_envs][N][slots]  'Requested_SOC' */
    const int32_t *arrivals;       /* [num_envs][N][max_vehicles]  'Arrivals' */
    const int32_t *departures;     /* [num_envs][N][max_vehicles]  'Departures' */
    const double *pv_ratio;        /* [num_envs] random_pv_shift_ratio */
} SngScenario;

typedef struct SngEnv SngEnv;
typedef struct SngGraph SngGraph;

int32_t sng_abi_version(void);
/* The library's build id: the first 12 hex digits of the SHA-256 of its sources (csrc/Makefile).  The
 * measurements committed under profiles/ name the build they were taken on by this id. */
const char *sng_build_id(void);

/* Fill `cfg` with the reference's defaults (N=8, '1h', b-pv, bounded, sparse). */
void sng_config_defaults(SngConfig *cfg);

/* SmartNanogridEnv.__init__ (smart_nanogrid_environment.py:32-120) for num_envs
 * independent environments on HIP device `device`.  Builds the PV/price tables
 * (pv_system_manager.py:10-91, accountant.py:48-101), allocates device state.
 * The BESS starts at bess_initial_soc and, as in the reference, is NOT reset by
 * sng_reset (central_management_system.py:93-94). */
int sng_create(const SngConfig *cfg, int device, int64_t num_envs, uint64_t seed, SngEnv **out);
void sng_destroy(SngEnv *env);
const char *sng_last_error(const SngEnv *env);
int sng_get_dims(const SngEnv *env, SngDims *out);
int sng_get_timestep(const SngEnv *env);

/* Global index of this handle's env 0 when one population of envs is sharded over several
 * GPUs/processes: env i then draws the streams of global env offset+i (reference RNG:
 * seed + offset + i; device RNG: hash-stream key of global env offset + i), so a sharded run reproduces the
 * single-GPU run bit for bit.  Call before reset. */
int sng_set_env_offset(SngEnv *env, int64_t offset);

/* SmartNanogridEnv.reset() (smart_nanogrid_environment.py:311-351) with generate_new_initial_values=True:
 * a new day for every env (charging_station.py:152-186), timestep 0, the t=0 observation into
 * obs[num_envs][obs_dim].  SNG_RNG_REFERENCE builds the days on host threads (the CPUs of
 * sched_getaffinity, capped by SNG_HOST_THREADS / OMP_NUM_THREADS) and uploads each chunk of envs
 * while the next is built. */
int sng_reset(SngEnv *env, int rng_mode, float *obs, void *stream);

/* reset(generate_new_initial_values=False) (smart_nanogrid_environment.py:347-357): replays the day this
 * handle last generated with sng_reset, as ChargingStation.load_initial_values (charging_station.py:
 * 119-136) re-reads the initial_values.json the generation wrote (:185-186): arrivals, departures, SoC,
 * occupancy and capacities as generated, Requested_SOC left at the 0 clear_initialisation_variables
 * (:138-150) wrote (so no vehicle penalty), a new PV ratio (:349 -- reference RNG: each env's Python
 * stream, after the owed day-end draw; device RNG: a replay stream), BESS carried over.
 * SNG_ERR_STATE if nothing was generated yet or an injected day (sng_reset_from_scenario) replaced it. */
int sng_reset_replay(SngEnv *env, float *obs, void *stream);

/* Start a day from given days in the reference's layout (host memory): the recorded KAT days, or
 * days exported with sng_get_scenario.  scenario->pv_ratio may be NULL: each env then draws its ratio
 * from its Python stream (smart_nanogrid_environment.py:349) as a reset does; the day-end draw the
 * last step owes (:181) is consumed either way once the streams exist. */
int sng_reset_from_scenario(SngEnv *env, const SngScenario *scenario, float *obs, void *stream);

/* Reseed: env i draws the streams of seed + global index i from the next reset on (reference RNG:
 * np.random.seed / random.seed of that value; device RNG: the hash streams of that seed, from day 0).
 * The loaded day stays loaded.  Synchronises `stream`. */
int sng_set_seed(SngEnv *env, uint64_t seed, void *stream);

/* SmartNanogridEnv.step(actions) (smart_nanogrid_environment.py:140-188) for every env:
 * one fused kernel.  reward = -total cost (f64), done = 1 at the end of the day.
 * `info` may be NULL.  Asynchronous on `stream`. */
int sng_step(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done,
             const SngInfo *info, void *stream);

/* sng_step with the actions in host memory and the outputs returned to host memory: the one-env gym path
   (smart_nanogrid_environment.py:140-188 as SB3's DummyVecEnv and solvers/evaluator.py:13-24 drive it: one
   step per call, results on the host).  actions [E][act_dim] f32, obs [E][obs_dim] f32, reward [E] f64,
   done [E] u8 and step_flags [E] u32 (each env's SNG_FLAG_* bits raised in this step; the sticky per-env flags
   and the flag summary are updated as by sng_step) are ordinary host memory of the caller.  The step kernel
   reads the actions from and writes the outputs to a per-handle block of mapped host memory, so the call is
   one kernel dispatch and one wait on `stream` (synchronous: returns when the outputs are in the caller's
   arrays).  info as sng_step, except that SngInfo.flags must be null.  Meant for small batches; a large one
   belongs on sng_step with device buffers. */
int sng_step_host(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done, uint32_t *step_flags,
                  const SngInfo *info, void *stream);

/* The kernel name (as rocprofv3 reports it) of the step kernel sng_step would launch next with this
 * `info` (NULL allowed): "void sng::step_lean_kernel<N, PK, REQ>" for stations of N in {1,2,4,8,10,16}
 * chargers stepped with one lane per env, no diagnostics, NumPy-2 promotion, a power-of-two dt,
 * bounded charging and no stochastic profiles; "void sng::step_kernel<NC, L, DIAG, FAST, PK>" otherwise. */
int sng_step_kernel_name(const SngEnv *env, const SngInfo *info, char *buf, int32_t len);

/* Sticky per-env error flags (SNG_FLAG_*), copied to host after the work queued on `stream`;
 * synchronises that stream only. */
int sng_read_errors(SngEnv *env, uint32_t *host_flags, int clear, void *stream);

/* State access (host arrays of num_envs doubles; [num_envs][N] for the vehicle SoC), ordered after the
 * work queued on `stream`; each synchronises that stream only.  Attribute reads of the reference's
 * components: battery_energy_storage_system.py:108-109, random_pv_shift_ratio, charger.py:16. */
int sng_get_battery_soc(SngEnv *env, double *host_soc, void *stream);
int sng_set_battery_soc(SngEnv *env, const double *host_soc, void *stream);
int sng_get_pv_ratio(SngEnv *env, double *host_ratio, void *stream);
int sng_get_vehicle_soc(SngEnv *env, double *host_soc, void *stream);   /* SOC[c, t] of the last step */
int sng_set_vehicle_soc(SngEnv *env, const double *host_soc, void *stream);

/* Checkpoint / resume of the whole simulation: EV SoC [N][E], BESS SoC and the
 * day's initial SoC (central_management_system.py:93-94), PV ratio, t = 0 penalty, sticky flags, the
 * loaded day (timeline, requested-SoC stream, profile factors), the timestep, the device day counter,
 * the replay bookkeeping, the reference RNG streams when they exist, and -- when episode_return is
 * given (device [num_envs] f64, e.g. SngInfo.episode_return) -- the running day returns.  The blob is
 * host memory of sng_state_size bytes; sng_set_state accepts only a blob of a handle with the same
 * configuration, num_envs and ABI.  Both synchronise `stream`. */
int sng_state_size(const SngEnv *env, int with_episode_return, size_t *bytes);
int sng_get_state(SngEnv *env, void *host_buf, size_t bytes, const double *episode_return, void *stream);
int sng_set_state(SngEnv *env, const void *host_buf, size_t bytes, double *episode_return, void *stream);

/* The current day of envs [first, first + count) in the reference's initial_values.json layout
 * (ChargingStation.generated_initial_values_json, charging_station.py:164-191), decoded from the device
 * timeline -- for host-generated, device-generated and injected days alike.
 * soc / occupancy / capacity / requested_soc: host [count][N][slots]; arrivals / departures: host
 * [count][N][max_vehicles], -1 padded (n_vehicles[count][N] holds the full counts); pv_ratio: [count].
 * 'SOC' holds the arrival SoCs and the recorded SOC[c, t] of empty chargers (the slots a step
 * reads); Requested_SOC is exact when requested SoC is enabled or any penalised value differs
 * from 1.0, and 1.0 on occupied slots otherwise (0 everywhere on a replayed day).  Valid after a reset
 * until the next reset; synchronises `stream`. */
int sng_get_scenario(SngEnv *env, int64_t first, int64_t count, int32_t max_vehicles, double *soc,
                     double *occupancy, double *capacity, double *requested_soc, int32_t *arrivals,
                     int32_t *departures, int32_t *n_vehicles, double *pv_ratio, void *stream);

/* Constant tables as built at create (host copies; n = 2*T). */
int sng_get_tables(const SngEnv *env, double *irr, double *irr_max, double *pv_power, double *price,
                   double *price_max, int32_t *n);

/* `days` full days captured as one hipGraph: ([device-RNG reset] + T fused steps) x days.
 * actions holds T consecutive [num_envs][act_dim] blocks (reused every day); obs/reward/done
 * are overwritten every step; info may be NULL.  Replays draw new days each time.
 * flags: SNG_GRAPH_*; days > 1 needs SNG_GRAPH_RESET.
 * day_returns (device [days][num_envs] f64, may be NULL): day d's returns accumulate into row
 * d instead of info->episode_return, so a replay leaves every day's returns for one
 * collective per replay (bench.py gathers them over RCCL while the next replay runs).
 * Without SNG_GRAPH_RESET the graph steps the day that is loaded at launch, from t = 0: device-RNG days,
 * host-RNG / injected days and replayed days are stepped with different encodings (sng_layout.h:
 * packed records, requested-SoC stream, cleared Requested_SOC, day-counter ownership), so launching a
 * steps-only graph over a day of another encoding than at capture, or after t = 0, fails with
 * SNG_ERR_STATE. */
#define SNG_GRAPH_RESET 1   /* start every day with a device-RNG reset */
int sng_graph_create(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done,
                     const SngInfo *info, int flags, int32_t days, double *day_returns, SngGraph **out);
int sng_graph_launch(SngGraph *graph, void *stream);
/* Kernel-time probe: runs `days` device-RNG days eagerly (as the graph does) and returns the
 * device time (ms) of every step kernel, ms[days*T], from HIP start/stop events attached to
 * each dispatch (hipExtLaunchKernel: the dispatch's own begin/end timestamps), and, when reset_ms
 * is not NULL, of every day's device reset, reset_ms[days] (the one-launch generator the same way;
 * wide stations' generator + profile + observe0 launches between recorded events).  ms = NULL: the
 * days are launched without per-dispatch events (back to back, for a caller's own timing).  Synchronises. */
int sng_time_step_kernels(SngEnv *env, const float *actions, float *obs, double *reward, uint8_t *done,
                          const SngInfo *info, int32_t days, float *ms, float *reset_ms, void *stream);
void sng_graph_destroy(SngGraph *graph);

/* Host-only entry points (no GPU needed): the reference-RNG scenario generator, for
 * checking against numpy/Python streams on CPU.  Outputs in SngScenario layout for
 * `num_envs` envs seeded seed+i; `episode` = number of days already drawn. */
int sng_host_generate_scenarios(const SngConfig *cfg, int64_t num_envs, uint64_t seed, int32_t episodes,
                                double *soc, double *occupancy, double *capacity, double *requested_soc,
                                int32_t *arrivals, int32_t *departures, int32_t max_vehicles,
                                double *pv_ratio);

/* Host threads the reference-RNG generator and the scenario encoder use (see sng_reset). */
int32_t sng_host_threads(void);

/* The device day counter: the number of device-RNG days this handle has started (the next device
 * reset draws day *out).  Synchronises `stream`. */
int sng_get_day_counter(SngEnv *env, uint64_t *out, void *stream);

/* Diagnostics: the measured bandwidth ceiling of device `device` for a step-sized launch.  One float4
 * copy kernel reads read_bytes and writes write_bytes (nontemporal stores, the step kernel's policy) per
 * dispatch; *dispatch_us = mean device time of `reps` dispatches each between its own start/stop events,
 * *back_to_back_us = mean start-to-start time of `reps` dispatches queued back to back (as a graph runs
 * them).  Allocates and frees its buffers; synchronises `stream`.  No reference counterpart. */
int sng_bandwidth_probe(int device, int64_t read_bytes, int64_t write_bytes, int32_t reps, float *dispatch_us,
                        float *back_to_back_us, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Multi-GPU exchange: one process per GPU, each with its contiguous env shard
 * (sng_set_env_offset); once per simulated day the per-env returns are all-gathered over RCCL
 * (xGMI within a node).  No per-step communication.  RCCL is loaded at the first call
 * (dlopen librccl.so.1).  Rank 0 makes the id with sng_comm_unique_id and hands it to every rank
 * (file, socket, MPI ...); each rank then calls sng_comm_create with it. */
#define SNG_COMM_ID_BYTES 128
typedef struct SngComm SngComm;
int sng_comm_unique_id(uint8_t *id /* [SNG_COMM_ID_BYTES] */);
int sng_comm_create(int device, int nranks, int rank, const uint8_t *id, SngComm **out);
/* local: device [count] f64 of this rank; global: device [nranks * count] f64, rank-major (= global
 * env order for equal contiguous shards).  Asynchronous on `stream`. */
int sng_allgather_returns(SngComm *comm, const double *local, double *global, int64_t count, void *stream);
void sng_comm_destroy(SngComm *comm);
const char *sng_comm_last_error(const SngComm *comm);   /* NULL: the calling thread's last create error */

#ifdef __cplusplus
}
#endif

#endif /* SNG_H */
