// sng_diag_hooks.h -- the diagnostic hooks of sng_kernels.hip.  In libsng.so every hook is empty.
//
// The diagnostic builds are separate translation units under tools/diag/ (never shipped): they define
// SNG_DIAG_STAMPS or SNG_DIAG_MEMFLOOR and then #include sng_kernels.hip, so the product source carries
// no A/B or diagnostic conditionals of its own.
//   SNG_DIAG_STAMPS   per-wave s_memrealtime stamps (100 MHz) at the step kernels' phase boundaries, kept
//                     in registers (no wait of their own) and written by each workgroup's first lane at the
//                     end: g_stamps[block * 8 + k] (tools/stamps.py).  SNG_WSTAMP_DECL declares the stamp
//                     array (a local or a member), SNG_WSTAMP(k) takes stamp k, SNG_WSTAMP_FLUSH writes them.
//   SNG_DIAG_MEMFLOOR the step kernels' loads and stores with trivial per-charger arithmetic: the timing
//                     floor of the data layout (tools/gpu_session.sh memfloor)
#pragma once

#if defined(SNG_DIAG_STAMPS)
__device__ unsigned long long *g_stamps;
#define SNG_WSTAMP_DECL unsigned long long stamp_[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define SNG_WSTAMP(k) stamp_[k] = __builtin_amdgcn_s_memrealtime()
// accumulating phase timers (ref_day2_kernel): t = SNG_WNOW(); ...; SNG_WACC(k, t) adds the elapsed ticks
#define SNG_WNOW() __builtin_amdgcn_s_memrealtime()
#define SNG_WACC(k, t0) stamp_[k] += __builtin_amdgcn_s_memrealtime() - (t0)
// slots 0..n-1 the stamps, slot 6 the XCC id (HW_REG_XCC_ID), slot 7 HW_REG_HW_ID (CU, SE, SIMD, wave slot)
#define SNG_WSTAMP_FLUSH(arr, n)                                                                       \
    do {                                                                                               \
        if (threadIdx.x == 0 && g_stamps) {                                                            \
            for (int i_ = 0; i_ < (n); ++i_) g_stamps[(size_t)blockIdx.x * 8 + i_] = (arr)[i_];       \
            g_stamps[(size_t)blockIdx.x * 8 + 6] = __builtin_amdgcn_s_getreg((3 << 11) | 20);          \
            g_stamps[(size_t)blockIdx.x * 8 + 7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);          \
        }                                                                                              \
    } while (0)
// one slot of record idx (8 slots per record) written by thread tid of the workgroup: a kernel with several
// records per workgroup (ref_day2_kernel: one per group of envs) or several wavefronts per record
#define SNG_WSTAMP_PUT(slot, v, idx, tid)                                                        \
    do {                                                                                         \
        if ((int)threadIdx.x == (tid) && g_stamps) g_stamps[(size_t)(idx) * 8 + (slot)] = (v);   \
    } while (0)
#define SNG_DIAG_SET_STAMPS                                                                         \
    extern "C" int sng_debug_set_stamps(unsigned long long *dev_ptr) {                              \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -1; \
    }
#else
#define SNG_WSTAMP_DECL [[maybe_unused]] unsigned char stamp_unused_
#define SNG_WSTAMP(k) \
    do {              \
    } while (0)
#define SNG_WSTAMP_FLUSH(arr, n) \
    do {                         \
    } while (0)
#define SNG_WSTAMP_PUT(slot, v, idx, tid) \
    do {                                  \
    } while (0)
#define SNG_WNOW() 0ull
#define SNG_WACC(k, t0) \
    do {                \
    } while (0)
#define SNG_DIAG_SET_STAMPS
#endif

#if defined(SNG_DIAG_MEMFLOOR)
// charger_step's body replaced: same inputs and outputs, trivial arithmetic
#define SNG_DIAG_CHARGER(o, aux, run, a) \
    do {                                 \
        (o).q = 0.0;                     \
        (o).pw = (aux) + (double)(a);    \
        (o).soc = (run) + (aux);         \
        (o).nx = 0u;                     \
        (o).fl = 0u;                     \
        return (o);                      \
    } while (0)
#else
#define SNG_DIAG_CHARGER(o, aux, run, a) \
    do {                                 \
    } while (0)
#endif
