// What does a dependent kernel dispatch cost below HIP?  A chain of kernel dispatch packets written straight
// into an HSA (AQL) queue, each with the barrier bit (it starts after the previous one completes, as a
// day's steps must), for several acquire / release fence scopes; the time per packet is the chain's wall
// time / its length (one completion signal on the last packet, one doorbell per chain).  The same kernels
// through hipGraph measured 1.85 us per node (empty, 2,048 workgroups: tools/diag/kernarg_probe.hip).
//   make -C tools/diag aql_probe      Run (from the repository root): tools/diag/aql_probe [packets]
// Kernels: aql_probe_kernels.co (k_empty; k_copy, 16 B in and out per lane), 2,048 workgroups of 64.
// Scopes: sys = system (HIP's default for a kernel whose results the host may read), agt = agent, none
// (valid only for a kernel whose results the next one does not read: the lower bound of the packet).
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define HK(x)                                                                        \
    do {                                                                             \
        hsa_status_t s_ = (x);                                                       \
        if (s_ != HSA_STATUS_SUCCESS) {                                              \
            const char *m_ = nullptr;                                                \
            hsa_status_string(s_, &m_);                                              \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?"); \
            std::exit(1);                                                            \
        }                                                                            \
    } while (0)

static hsa_agent_t g_gpu{0}, g_cpu{0};
static hsa_region_t g_kernarg{0};
static hsa_amd_memory_pool_t g_devpool{0};

static hsa_status_t find_agents(hsa_agent_t a, void *) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_kernarg(hsa_region_t r, void *) {
    hsa_region_segment_t seg;
    hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg);
    if (seg != HSA_REGION_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_REGION_GLOBAL_FLAG_KERNARG) && g_kernarg.handle == 0) g_kernarg = r;
    return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_devpool(hsa_amd_memory_pool_t p, void *) {
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && g_devpool.handle == 0) g_devpool = p;
    return HSA_STATUS_SUCCESS;
}

struct Kernel {
    uint64_t object = 0;
    uint32_t kernarg_size = 0, group = 0, priv = 0;
};

static Kernel get_kernel(hsa_executable_t ex, const char *name) {
    hsa_executable_symbol_t sym;
    HK(hsa_executable_get_symbol_by_name(ex, name, &g_gpu, &sym));
    Kernel k;
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg_size));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
    HK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
    return k;
}

static uint16_t header(bool barrier, hsa_fence_scope_t acq, hsa_fence_scope_t rel) {
    return (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                      ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                      (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                      (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
}

// n dependent dispatches of kernel k; the last one releases at system scope and signals; returns us per packet
static hsa_signal_t g_each{0};   // a completion signal on every packet (the `sig` configurations)
static double chain(hsa_queue_t *q, const Kernel &k, void *kernarg, int n, hsa_fence_scope_t acq,
                    hsa_fence_scope_t rel, bool barrier, hsa_signal_t done, bool each = false) {
    hsa_signal_store_screlease(done, 1);
    auto *pkts = reinterpret_cast<hsa_kernel_dispatch_packet_t *>(q->base_address);
    const uint32_t mask = q->size - 1;
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t idx = hsa_queue_add_write_index_relaxed(q, (uint64_t)n);
    const uint64_t first = idx;
    for (int i = 0; i < n; ++i, ++idx) {
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        }
        hsa_kernel_dispatch_packet_t *p = &pkts[idx & mask];
        std::memset(reinterpret_cast<char *>(p) + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = 64;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = 2048 * 64;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->private_segment_size = k.priv;
        p->group_segment_size = k.group;
        p->kernel_object = k.object;
        p->kernarg_address = kernarg;
        const bool last = i == n - 1;
        p->completion_signal = last ? done : each ? g_each : hsa_signal_t{0};
        const uint16_t h = last ? header(true, acq, HSA_FENCE_SCOPE_SYSTEM) : header(barrier, acq, rel);
        const uint32_t word = (uint32_t)h | ((uint32_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16);
        __atomic_store_n(reinterpret_cast<uint32_t *>(p), word, __ATOMIC_RELEASE);
    }
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(first + n - 1));
    while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {
    }
    const auto t1 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / n;
}

// Coherence mode: iterations of (check the previous value through one workgroup mapping, write a new value,
// check it through another mapping) as one chain of dependent packets with the given inner fence scopes; the
// count of words a check found stale.  A stale word means the inner fences do not make one kernel's stores
// visible to the next kernel's loads.
struct WriteArgs {
    unsigned *buf;
    unsigned seq;
    int pol;
};
struct CheckArgs {
    const unsigned *buf;
    unsigned want, mul, add;
    unsigned long long *errors;
    unsigned nblk;
};
static unsigned long long coherence(hsa_queue_t *q, const Kernel &kw, const Kernel &kc, int iters, int pol,
                                    hsa_fence_scope_t acq, hsa_fence_scope_t rel, hsa_signal_t done) {
    const unsigned nblk = 2048;
    unsigned *buf = nullptr;
    unsigned long long *errors = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_devpool, (size_t)nblk * 64 * 4, 0, reinterpret_cast<void **>(&buf)));
    HK(hsa_amd_memory_pool_allocate(g_devpool, 64, 0, reinterpret_cast<void **>(&errors)));
    HK(hsa_amd_memory_fill(buf, 0, nblk * 64));
    HK(hsa_amd_memory_fill(errors, 0, 16));
    const int n = 3 * iters;
    const size_t slot = 64;
    std::vector<unsigned char> host((size_t)n * slot, 0);
    for (int k = 0; k < iters; ++k) {
        CheckArgs before{buf, (unsigned)k, 2u * (unsigned)(k % 997) + 1u, (unsigned)k * 97u, errors, nblk};
        WriteArgs w{buf, (unsigned)(k + 1), pol};
        CheckArgs after{buf, (unsigned)(k + 1), 2u * (unsigned)((k * 7 + 3) % 991) + 1u, (unsigned)k * 31u + 5u, errors,
                        nblk};
        std::memcpy(&host[(size_t)(3 * k) * slot], &before, sizeof(before));
        std::memcpy(&host[(size_t)(3 * k + 1) * slot], &w, sizeof(w));
        std::memcpy(&host[(size_t)(3 * k + 2) * slot], &after, sizeof(after));
    }
    unsigned char *ka = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_devpool, host.size(), 0, reinterpret_cast<void **>(&ka)));
    HK(hsa_memory_copy(ka, host.data(), host.size()));
    hsa_signal_store_screlease(done, 1);
    auto *pkts = reinterpret_cast<hsa_kernel_dispatch_packet_t *>(q->base_address);
    const uint32_t mask = q->size - 1;
    uint64_t idx = hsa_queue_add_write_index_relaxed(q, (uint64_t)n);
    const uint64_t first = idx;
    for (int i = 0; i < n; ++i, ++idx) {
        while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
            hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(idx - 1));
        }
        const Kernel &k = (i % 3 == 1) ? kw : kc;
        hsa_kernel_dispatch_packet_t *p = &pkts[idx & mask];
        std::memset(reinterpret_cast<char *>(p) + 4, 0, sizeof(*p) - 4);
        p->workgroup_size_x = 64;
        p->workgroup_size_y = 1;
        p->workgroup_size_z = 1;
        p->grid_size_x = nblk * 64;
        p->grid_size_y = 1;
        p->grid_size_z = 1;
        p->private_segment_size = k.priv;
        p->group_segment_size = k.group;
        p->kernel_object = k.object;
        p->kernarg_address = ka + (size_t)i * slot;
        const bool last = i == n - 1;
        p->completion_signal = last ? done : hsa_signal_t{0};
        const uint16_t h = last ? header(true, acq, HSA_FENCE_SCOPE_SYSTEM)
                                : header(true, i == 0 ? HSA_FENCE_SCOPE_SYSTEM : acq, rel);
        const uint32_t word = (uint32_t)h | ((uint32_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS) << 16);
        __atomic_store_n(reinterpret_cast<uint32_t *>(p), word, __ATOMIC_RELEASE);
    }
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)(first + n - 1));
    while (hsa_signal_wait_scacquire(done, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {
    }
    unsigned long long errs = 0;
    HK(hsa_memory_copy(&errs, errors, sizeof(errs)));
    hsa_amd_memory_pool_free(ka);
    hsa_amd_memory_pool_free(buf);
    hsa_amd_memory_pool_free(errors);
    return errs;
}

int main(int argc, char **argv) {
    const bool coh = argc > 1 && std::strcmp(argv[1], "coherence") == 0;
    const int n = (argc > 1 && !coh) ? std::atoi(argv[1]) : 1200;
    const char *co_path = (argc > 2 && !coh) ? argv[2] : "tools/diag/aql_probe_kernels.co";
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    if (!g_gpu.handle) {
        std::fprintf(stderr, "no GPU agent\n");
        return 1;
    }
    HK(hsa_agent_iterate_regions(g_gpu, find_kernarg, nullptr));
    HK(hsa_amd_agent_iterate_memory_pools(g_gpu, find_devpool, nullptr));
    std::ifstream f(co_path, std::ios::binary);
    if (!f) {
        std::fprintf(stderr, "cannot read %s\n", co_path);
        return 1;
    }
    std::string blob((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    hsa_code_object_reader_t rd;
    HK(hsa_code_object_reader_create_from_memory(blob.data(), blob.size(), &rd));
    hsa_executable_t ex;
    HK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
    HK(hsa_executable_load_agent_code_object(ex, g_gpu, rd, nullptr, nullptr));
    HK(hsa_executable_freeze(ex, nullptr));
    const Kernel ke = get_kernel(ex, "k_empty.kd"), kc = get_kernel(ex, "k_copy.kd");

    hsa_queue_t *q;
    HK(hsa_queue_create(g_gpu, 4096, HSA_QUEUE_TYPE_SINGLE, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    hsa_signal_t done;
    HK(hsa_signal_create(1, 0, nullptr, &done));
    if (coh) {
        const int iters = argc > 2 ? std::atoi(argv[2]) : 300;
        const Kernel kw = get_kernel(ex, "k_write.kd"), kk = get_kernel(ex, "k_check.kd");
        struct {
            const char *name;
            hsa_fence_scope_t acq, rel;
        } sc[] = {{"acq agent, rel agent", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT},
                  {"acq agent, rel none ", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_NONE},
                  {"acq none,  rel agent", HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT},
                  {"acq none,  rel none ", HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE}};
        std::printf("coherence: %d x (check old, write new, check new), 2,048 x 64 words; stale words counted\n", iters);
        for (int rep = 0; rep < 3; ++rep)
            for (int pol = 0; pol < 2; ++pol)
                for (auto &c : sc) {
                    const unsigned long long e = coherence(q, kw, kk, iters, pol, c.acq, c.rel, done);
                    std::printf("rep %d  %s  %s store  stale words %llu of %llu\n", rep, c.name, pol ? "nt   " : "plain",
                                e, (unsigned long long)iters * 2 * 2048 * 64);
                    std::fflush(stdout);
                }
        HK(hsa_signal_destroy(done));
        HK(hsa_queue_destroy(q));
        return 0;
    }

    // device buffers for k_copy (2,048 x 64 lanes x 16 B each way)
    const size_t bytes = (size_t)2048 * 64 * 16;
    void *in = nullptr, *out = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_devpool, bytes, 0, &in));
    HK(hsa_amd_memory_pool_allocate(g_devpool, bytes, 0, &out));
    // kernarg blocks (zeroed; k_copy's two pointers first)
    void *ka_e = nullptr, *ka_c = nullptr;
    HK(hsa_memory_allocate(g_kernarg, ke.kernarg_size ? ke.kernarg_size : 64, &ka_e));
    HK(hsa_memory_allocate(g_kernarg, kc.kernarg_size, &ka_c));
    std::memset(ka_e, 0, ke.kernarg_size ? ke.kernarg_size : 64);
    std::memset(ka_c, 0, kc.kernarg_size);
    void *ptrs[2] = {in, out};
    std::memcpy(ka_c, ptrs, sizeof(ptrs));
    // the same arguments in device memory (as HIP keeps them): the kernarg region is host memory, and a
    // wavefront's argument load from it crosses PCIe after every acquire
    void *ka_cd = nullptr;
    HK(hsa_amd_memory_pool_allocate(g_devpool, 4096, 0, &ka_cd));
    HK(hsa_memory_copy(ka_cd, ka_c, kc.kernarg_size));
    HK(hsa_amd_memory_fill(in, 0, bytes / 4));
    HK(hsa_amd_memory_fill(out, 0, bytes / 4));
    HK(hsa_signal_create(1 << 30, 0, nullptr, &g_each));
    for (int w = 0; w < 20; ++w)   // warm the copy (pages, clocks) before anything is timed
        chain(q, kc, ka_cd, n, HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT, true, done);

    struct Cfg {
        const char *name;
        hsa_fence_scope_t acq, rel;
        bool barrier, each;
    } cfgs[] = {{"barrier acq sys  rel sys ", HSA_FENCE_SCOPE_SYSTEM, HSA_FENCE_SCOPE_SYSTEM, true},
                {"barrier acq agt  rel agt ", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT, true},
                {"barrier agt/agt + signal ", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_AGENT, true, true},
                {"barrier agt/sys + signal ", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_SYSTEM, true, true},
                {"barrier acq agt  rel sys ", HSA_FENCE_SCOPE_AGENT, HSA_FENCE_SCOPE_SYSTEM, true},
                {"barrier acq none rel agt ", HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_AGENT, true},
                {"barrier acq none rel none", HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE, true},
                {"no barrier, none / none  ", HSA_FENCE_SCOPE_NONE, HSA_FENCE_SCOPE_NONE, false}};
    std::printf("%d dispatches per chain, 2,048 workgroups of 64; us per dispatch (best of 5)\n", n);
    for (int pass = 0; pass < 2; ++pass)
        for (const Cfg &c : cfgs)
            for (int kk = 0; kk < 3; ++kk) {
                const Kernel &k = kk ? kc : ke;
                void *ka = kk == 2 ? ka_cd : kk ? ka_c : ka_e;
                double best = 1e30;
                for (int r = 0; r < 6; ++r) {
                    const double us = chain(q, k, ka, n, c.acq, c.rel, c.barrier, done, c.each);
                    if (r > 0 && us < best) best = us;   // the first chain warms the queue
                }
                std::printf("pass %d  %s  %-12s %.3f\n", pass, c.name, kk == 2 ? "copy dev-ka" : kk ? "copy host-ka" : "empty", best);
                std::fflush(stdout);
            }
    HK(hsa_signal_destroy(done));
    HK(hsa_signal_destroy(g_each));
    HK(hsa_queue_destroy(q));
    hsa_memory_free(ka_e);
    hsa_memory_free(ka_c);
    hsa_amd_memory_pool_free(ka_cd);
    hsa_amd_memory_pool_free(in);
    hsa_amd_memory_pool_free(out);
    HK(hsa_executable_destroy(ex));
    HK(hsa_code_object_reader_destroy(rd));
    HK(hsa_shut_down());
    return 0;
}
