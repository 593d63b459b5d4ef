// marf_comm.hip -- the MLP-gradient exchange of the patch-sharded step over RCCL.
//
// The reference is single-GPU (options.py:117-120); sharding the patches over the GPUs of a node
// leaves one exchange per step: the sum of the shared MLP gradient over ranks (each rank's warp rows
// stay local).  This unit talks to RCCL directly (librccl.so from ROCm, opened at first use, so the
// library still loads where RCCL is absent) for hosts that do not bring torch.distributed:
//   marf_comm_unique_id / marf_comm_create / marf_comm_destroy   -- one communicator per rank
//   marf_allreduce_grads         -- one in-place fp32 sum of a flat gradient on the caller's stream
//   marf_allreduce_grads_layers  -- the same per layer: each layer's slice is summed on the
//                                   communicator's own stream as soon as marf_step_backward_ev
//                                   marked it final, so the exchange of the layers that finish first
//                                   overlaps the weight gradients of the others; the caller's stream
//                                   waits for the last one.
#include <dlfcn.h>
#include <string.h>

#include <mutex>

#include <rccl/rccl.h>

#include "../../include/marf.h"

namespace {

struct Rccl {
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
        r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
        r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
        r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
        r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
        r.ok = r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.error_string;
    });
    return r;
}

}  // namespace

struct marf_comm {
    ncclComm_t comm = nullptr;
    int device = 0, nranks = 1, rank = 0;
    hipStream_t side = nullptr;      // the per-layer exchanges
    hipEvent_t joined = nullptr;     // the last of them, for the caller's stream to wait on
    hipEvent_t entry = nullptr;      // the caller's stream at the call (stands in for a NULL layer event)
};

// (marf_abi.hip's error slot)
extern "C" int marf_set_error(int code, const char* msg);

static int rccl_fail(const char* what, ncclResult_t r) {
    char buf[256];
    snprintf(buf, sizeof buf, "%s: %s", what, rccl().error_string ? rccl().error_string(r) : "RCCL error");
    return marf_set_error(MARF_ERR_HIP, buf);
}

extern "C" {

int marf_comm_unique_id(void* out, size_t cap) {
    if (!out || cap < sizeof(ncclUniqueId)) return marf_set_error(MARF_ERR_INVALID, "comm_unique_id: buffer < 128 B");
    if (!rccl().ok) return marf_set_error(MARF_ERR_UNSUPPORTED, "comm_unique_id: librccl.so not found");
    ncclUniqueId id;
    ncclResult_t r = rccl().get_unique_id(&id);
    if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
    memcpy(out, &id, sizeof id);
    return MARF_OK;
}

int marf_comm_create(const void* unique_id, int nranks, int rank, int device, marf_comm** out) {
    if (!unique_id || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return marf_set_error(MARF_ERR_INVALID, "comm_create: bad arguments");
    if (!rccl().ok) return marf_set_error(MARF_ERR_UNSUPPORTED, "comm_create: librccl.so not found");
    // the communicator is created on `device`; the calling thread's current device is restored on
    // every path (no hidden global side effect)
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) return marf_set_error(MARF_ERR_HIP, "comm_create: hipGetDevice");
    struct Restore {
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{prev};
    if (hipSetDevice(device) != hipSuccess) return marf_set_error(MARF_ERR_HIP, "comm_create: hipSetDevice");
    marf_comm* c = new marf_comm;
    c->device = device;
    c->nranks = nranks;
    c->rank = rank;
    ncclUniqueId id;
    memcpy(&id, unique_id, sizeof id);
    ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, id, rank);
    if (r != ncclSuccess) {
        delete c;
        return rccl_fail("ncclCommInitRank", r);
    }
    if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->joined, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->entry, hipEventDisableTiming) != hipSuccess) {
        rccl().comm_destroy(c->comm);
        if (c->joined) (void)hipEventDestroy(c->joined);
        if (c->side) (void)hipStreamDestroy(c->side);
        delete c;
        return marf_set_error(MARF_ERR_HIP, "comm_create: stream / event");
    }
    *out = c;
    return MARF_OK;
}

void marf_comm_destroy(marf_comm* c) {
    if (!c) return;
    if (c->side) (void)hipStreamSynchronize(c->side);
    if (c->comm) rccl().comm_destroy(c->comm);
    if (c->joined) (void)hipEventDestroy(c->joined);
    if (c->entry) (void)hipEventDestroy(c->entry);
    if (c->side) (void)hipStreamDestroy(c->side);
    delete c;
}

int marf_allreduce_grads(marf_comm* c, float* d_flat, size_t n, void* stream) {
    if (!c || (n && !d_flat)) return marf_set_error(MARF_ERR_INVALID, "allreduce_grads: bad arguments");
    if (!n) return MARF_OK;
    ncclResult_t r = rccl().all_reduce(d_flat, d_flat, n, ncclFloat32, ncclSum, c->comm, (hipStream_t)stream);
    return r == ncclSuccess ? MARF_OK : rccl_fail("ncclAllReduce", r);
}

// A NULL entry of layer_events (a layer the backward did not mark) waits for everything queued on
// the caller's stream before this call instead.  If a collective fails after others were queued,
// the caller's stream is still joined to the side stream before the error returns, but the ranks'
// collective sequences may now disagree: destroy the communicator after an error (include/marf.h).
int marf_allreduce_grads_layers(marf_comm* c, const marf_net* net, float* d_dparams, void* const* layer_events,
                                void* stream) {
    if (!c || !net || !d_dparams || !layer_events) return marf_set_error(MARF_ERR_INVALID, "allreduce_grads_layers: NULL");
    const int nl = marf_net_layer_count(net);
    hipStream_t s = (hipStream_t)stream;
    bool entry_recorded = false;
    int rc = MARF_OK, queued = 0;
    // the order marf_step_backward_ev finishes them: last layer first
    for (int l = nl - 1; l >= 0 && rc == MARF_OK; --l) {
        long long off = 0, len = 0;
        if (marf_net_layer_span(net, l, &off, &len) != MARF_OK) {
            rc = MARF_ERR_INVALID;
            break;
        }
        hipEvent_t ev = (hipEvent_t)layer_events[l];
        if (!ev) {
            if (!entry_recorded && hipEventRecord(c->entry, s) != hipSuccess) {
                rc = marf_set_error(MARF_ERR_HIP, "allreduce_grads_layers: record");
                break;
            }
            entry_recorded = true;
            ev = c->entry;
        }
        if (hipStreamWaitEvent(c->side, ev, 0) != hipSuccess) {
            rc = marf_set_error(MARF_ERR_HIP, "allreduce_grads_layers: wait");
            break;
        }
        ncclResult_t r = rccl().all_reduce(d_dparams + off, d_dparams + off, (size_t)len, ncclFloat32, ncclSum, c->comm,
                                           c->side);
        if (r != ncclSuccess) rc = rccl_fail("ncclAllReduce (layer)", r);
        else ++queued;
    }
    if (rc != MARF_OK && queued == 0) return rc;  // nothing queued: the caller's stream is untouched
    // join (also after a failure, so that the caller's stream never runs ahead of queued collectives)
    if (hipEventRecord(c->joined, c->side) != hipSuccess || hipStreamWaitEvent(s, c->joined, 0) != hipSuccess)
        return rc != MARF_OK ? rc : marf_set_error(MARF_ERR_HIP, "allreduce_grads_layers: join");
    return rc;
}

}  // extern "C"
