// sng_comm.cpp -- the multi-GPU exchange of the C ABI (include/sng.h): one RCCL
// communicator per process (one process per GPU, as bench.py runs) and the all-gather of the
// per-env day returns of every rank's contiguous env shard, so a host without torch.distributed
// (C, C++, another language over the C ABI) has the same multi-GPU path.
//
// RCCL is loaded on first use with dlopen("librccl.so.1") and called through dlsym'd pointers:
// libsng.so does not link it, and in a process that already holds RCCL (torch) the loader hands
// back that same copy, so the two share one library.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "sng.h"

static_assert(SNG_COMM_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");

namespace {

thread_local std::string g_comm_error;

struct Rccl {
    void *handle = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char *name : {"librccl.so.1", "librccl.so"}) {
            r.handle = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.handle) break;
        }
        if (!r.handle) {
            r.error = std::string("cannot load RCCL (librccl.so.1): ") + dlerror();
            return;
        }
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(r.handle, "ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(r.handle, "ncclCommInitRank"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(r.handle, "ncclAllGather"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(r.handle, "ncclCommDestroy"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(r.handle, "ncclGetErrorString"));
        if (!r.get_unique_id || !r.init_rank || !r.all_gather || !r.destroy || !r.error_string)
            r.error = "RCCL is missing a symbol this library needs";
    });
    return r;
}

}  // namespace

struct SngComm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    std::string err;
};

namespace {

int comm_fail(SngComm *c, int code, const std::string &msg) {
    if (c) c->err = msg; else g_comm_error = msg;
    return code;
}

std::string nccl_msg(const char *what, ncclResult_t r) {
    return std::string(what) + ": " + rccl().error_string(r);
}

}  // namespace

extern "C" {

const char *sng_comm_last_error(const SngComm *comm) { return comm ? comm->err.c_str() : g_comm_error.c_str(); }

int sng_comm_unique_id(uint8_t *id) {
    if (!id) return comm_fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "null id");
    const Rccl &r = rccl();
    if (!r.error.empty()) return comm_fail(nullptr, SNG_ERR_UNSUPPORTED, r.error);
    ncclUniqueId uid;
    ncclResult_t e = r.get_unique_id(&uid);
    if (e != ncclSuccess) return comm_fail(nullptr, SNG_ERR_HIP, nccl_msg("ncclGetUniqueId", e));
    std::memcpy(id, uid.internal, SNG_COMM_ID_BYTES);
    return SNG_OK;
}

int sng_comm_create(int device, int nranks, int rank, const uint8_t *id, SngComm **out) {
    if (!out || !id) return comm_fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return comm_fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "bad rank");
    const Rccl &r = rccl();
    if (!r.error.empty()) return comm_fail(nullptr, SNG_ERR_UNSUPPORTED, r.error);
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) return comm_fail(nullptr, SNG_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, SNG_COMM_ID_BYTES);
    SngComm *c = new SngComm();
    ncclResult_t e = r.init_rank(&c->comm, nranks, uid, rank);
    if (e != ncclSuccess) {
        delete c;
        return comm_fail(nullptr, SNG_ERR_HIP, nccl_msg("ncclCommInitRank", e));
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return SNG_OK;
}

int sng_allgather_returns(SngComm *comm, const double *local, double *global, int64_t count, void *stream) {
    if (!comm) return comm_fail(nullptr, SNG_ERR_INVALID_ARGUMENT, "null communicator");
    if (!local || !global || count < 1) return comm_fail(comm, SNG_ERR_INVALID_ARGUMENT, "bad buffers");
    hipError_t he = hipSetDevice(comm->device);
    if (he != hipSuccess) return comm_fail(comm, SNG_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
    ncclResult_t e = rccl().all_gather(local, global, (size_t)count, ncclFloat64, comm->comm, (hipStream_t)stream);
    if (e != ncclSuccess) return comm_fail(comm, SNG_ERR_HIP, nccl_msg("ncclAllGather", e));
    return SNG_OK;
}

void sng_comm_destroy(SngComm *comm) {
    if (!comm) return;
    if (comm->comm) (void)rccl().destroy(comm->comm);
    delete comm;
}

}  // extern "C"
