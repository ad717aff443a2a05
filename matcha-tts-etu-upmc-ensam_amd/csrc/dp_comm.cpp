// Data-parallel gradient exchange over RCCL (xGMI), callable from inside a captured HIP graph.
//
// The reference trains on one device (train.py:81-84); the north star shards utterances over the GPUs
// of a node with the gradient all-reduce overlapped with backward.  torch's ProcessGroupNCCL cannot be
// captured into a HIP graph on this stack (its watchdog queries events while the stream captures ->
// hipErrorStreamCaptureUnsupported, tools/graph_event_probe.py), and torch refuses external events on
// ROCm, so the training step's graph issues the bucket all-reduces itself: this file owns an RCCL
// communicator (one per process, ranks = torch.distributed ranks) and enqueues ncclAllReduce on a
// caller stream -- inside stream capture that becomes a graph node on a forked branch, so each bucket's
// reduction overlaps the rest of the backward when the graph replays.
//
// librccl is opened at run time (dlopen): the copy torch already loaded (soname librccl.so.1) is reused,
// so the process holds one RCCL; nothing links against it at build time.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <mutex>

#include "mtts_common.h"
#include "mtts_dp.h"

namespace {

struct Rccl {
    void *handle = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGetVersion) get_version = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
};

std::mutex g_mu;
Rccl g_rccl;

const Rccl *rccl() {
    std::lock_guard<std::mutex> lock(g_mu);
    if (g_rccl.handle) return &g_rccl;
    void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, if loaded
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        mtts::set_error("dp_comm: cannot dlopen librccl (%s)", dlerror());
        return nullptr;
    }
    Rccl r;
    r.handle = h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.get_version = reinterpret_cast<decltype(r.get_version)>(dlsym(h, "ncclGetVersion"));
    r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(h, "ncclCommCount"));
    r.comm_user_rank = reinterpret_cast<decltype(r.comm_user_rank)>(dlsym(h, "ncclCommUserRank"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string ||
        !r.comm_count || !r.comm_user_rank) {
        mtts::set_error("dp_comm: librccl lacks an entry point");
        return nullptr;
    }
    g_rccl = r;
    return &g_rccl;
}

int rccl_fail(const Rccl *r, ncclResult_t rc, const char *what) {
    mtts::set_error("dp_comm: %s failed: %s", what, r->error_string ? r->error_string(rc) : "?");
    return MTTS_ERR_HIP;
}

}  // namespace

extern "C" int mtts_dp_unique_id(void *id_out, size_t bytes) {
    MTTS_CHECK_ARG(id_out && bytes >= sizeof(ncclUniqueId), "dp_unique_id: need 128 bytes");
    const Rccl *r = rccl();
    if (!r) return MTTS_ERR_HIP;
    ncclUniqueId id;
    const ncclResult_t rc = r->get_unique_id(&id);
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclGetUniqueId");
    std::memcpy(id_out, &id, sizeof(id));
    return MTTS_OK;
}

extern "C" int mtts_dp_comm_init(const void *id, size_t bytes, int32_t nranks, int32_t rank, void **comm_out) {
    MTTS_CHECK_ARG(id && comm_out && bytes >= sizeof(ncclUniqueId) && nranks >= 1 && rank >= 0 && rank < nranks,
                   "dp_comm_init: bad args");
    const Rccl *r = rccl();
    if (!r) return MTTS_ERR_HIP;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t rc = r->comm_init_rank(&comm, nranks, uid, rank);  // on the caller's current device
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclCommInitRank");
    *comm_out = comm;
    return MTTS_OK;
}

extern "C" int mtts_dp_allreduce_f32(void *comm, float *buf, int64_t count, int32_t average, void *hip_stream) {
    MTTS_CHECK_ARG(comm && buf && count >= 0, "dp_allreduce_f32: bad args");
    if (count == 0) return MTTS_OK;
    const Rccl *r = rccl();
    if (!r) return MTTS_ERR_HIP;
    const ncclResult_t rc = r->all_reduce(buf, buf, (size_t)count, ncclFloat32, average ? ncclAvg : ncclSum,
                                          static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(hip_stream));
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclAllReduce");
    return MTTS_OK;
}

extern "C" int mtts_dp_comm_query(void *comm, int32_t *nranks_out, int32_t *rank_out) {
    MTTS_CHECK_ARG(comm && nranks_out && rank_out, "dp_comm_query: bad args");
    const Rccl *r = rccl();
    if (!r) return MTTS_ERR_HIP;
    int n = 0, me = 0;
    ncclResult_t rc = r->comm_count(static_cast<ncclComm_t>(comm), &n);
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclCommCount");
    rc = r->comm_user_rank(static_cast<ncclComm_t>(comm), &me);
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclCommUserRank");
    *nranks_out = n;
    *rank_out = me;
    return MTTS_OK;
}

extern "C" int mtts_dp_comm_destroy(void *comm) {
    if (!comm) return MTTS_OK;
    const Rccl *r = rccl();
    if (!r) return MTTS_ERR_HIP;
    const ncclResult_t rc = r->comm_destroy(static_cast<ncclComm_t>(comm));
    if (rc != ncclSuccess) return rccl_fail(r, rc, "ncclCommDestroy");
    return MTTS_OK;
}

extern "C" int mtts_dp_rccl_version(void) {
    const Rccl *r = rccl();
    int v = 0;
    if (!r || !r->get_version || r->get_version(&v) != ncclSuccess) return -1;
    return v;
}

// ------------------------------------------------------------------------------------------------
// Device-side progress markers for the host watchdog of the data-parallel bench: a coherent,
// host-mapped int32 array the host reads at any time without synchronising, written by a one-lane kernel that is
// stream-ordered and capturable -- inside the step's graph after each bucket's all-reduce (reducer stream) and at
// the end of the step (main stream).  Slot 0 = steps the device has completed (a device-side counter incremented
// by the step-end mark), slot s > 0 = steps * 256 + tag of the last mark on that slot (tag = bucket index + 1).
namespace {
struct Progress {
    int32_t *host = nullptr;  // hipHostMalloc(mapped | coherent): the watchdog reads it
    int32_t *dev = nullptr;   // device step counter
    int32_t nslots = 0;
};

// vector stores only (the store address is lane-dependent; one lane is active)
__global__ void progress_mark_kernel(int32_t *__restrict__ dev, int32_t *host, int32_t slot, int32_t tag) {
    const int l = threadIdx.x;
    if (l != 0) return;
    int32_t steps = dev[l];
    if (tag < 0) {
        steps += 1;
        dev[l] = steps;
        __hip_atomic_store(host + l, steps, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        __hip_atomic_store(host + slot + l, steps * 256 + tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
}  // namespace

extern "C" int mtts_dp_progress_create(int32_t nslots, void **handle_out, int32_t **host_out) {
    MTTS_CHECK_ARG(handle_out && host_out && nslots >= 1 && nslots <= 64, "dp_progress_create: bad args");
    Progress *pr = new Progress();
    pr->nslots = nslots;
    if (hipHostMalloc(reinterpret_cast<void **>(&pr->host), sizeof(int32_t) * nslots,
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipMalloc(reinterpret_cast<void **>(&pr->dev), sizeof(int32_t)) != hipSuccess ||
        hipMemset(pr->dev, 0, sizeof(int32_t)) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        if (pr->host) hipHostFree(pr->host);
        if (pr->dev) hipFree(pr->dev);
        delete pr;
        return mtts::fail(MTTS_ERR_HIP, "dp_progress_create: allocation failed");
    }
    std::memset(pr->host, 0, sizeof(int32_t) * nslots);
    *handle_out = pr;
    *host_out = pr->host;
    return MTTS_OK;
}

extern "C" int mtts_dp_progress_mark(void *handle, int32_t slot, int32_t tag, void *hip_stream) {
    Progress *pr = static_cast<Progress *>(handle);
    MTTS_CHECK_ARG(pr && slot >= 0 && slot < pr->nslots && (tag < 0 || slot > 0), "dp_progress_mark: bad args");
    hipLaunchKernelGGL(progress_mark_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(hip_stream), pr->dev,
                       pr->host, slot, tag);
    return mtts::check_launch("progress_mark_kernel");
}

extern "C" int mtts_dp_progress_destroy(void *handle) {
    Progress *pr = static_cast<Progress *>(handle);
    if (!pr) return MTTS_OK;
    hipDeviceSynchronize();
    hipHostFree(pr->host);
    hipFree(pr->dev);
    delete pr;
    return MTTS_OK;
}
