// comm.cpp -- the one collective of the multi-GPU path: RCCL all-reduce of small
// host vectors (per-unit row and byte counts, the step time), bound here so
// that a multi-rank run needs no PyTorch (bwtmi/comm.py does the rendezvous).
//
// The reference has no collective: its contig workers return through
// multiprocessing.Pool pickling (bwt.py:3894-3912).  Here every rank writes its
// own fold units into the shared output file at offsets from two sums over
// ranks (bwtmi/dist.py write_sharded), so the only data on the wire are those
// count vectors -- a latency-bound exchange over xGMI.
//
// librccl is opened with dlopen on first use: single-GPU runs never load it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>

#include "common.h"
#include "device.h"

namespace {

// types, enums and the id layout come from the image's own header; the
// functions are resolved with dlsym so single-GPU runs never load librccl
struct Rccl {
    void *h = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    static const char *open_error = nullptr;
    std::call_once(once, [] {
        for (const char *name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.h) break;
        }
        if (!r.h) {
            open_error = dlerror();   // read once: the call clears it
            return;
        }
        r.GetUniqueId = (decltype(r.GetUniqueId))dlsym(r.h, "ncclGetUniqueId");
        r.CommInitRank = (decltype(r.CommInitRank))dlsym(r.h, "ncclCommInitRank");
        r.AllReduce = (decltype(r.AllReduce))dlsym(r.h, "ncclAllReduce");
        r.CommDestroy = (decltype(r.CommDestroy))dlsym(r.h, "ncclCommDestroy");
        r.GetErrorString = (decltype(r.GetErrorString))dlsym(r.h, "ncclGetErrorString");
    });
    if (!r.h || !r.GetUniqueId || !r.CommInitRank || !r.AllReduce || !r.CommDestroy)
        bwtmi::fail(BWTMI_E_NODEVICE, "librccl could not be loaded: %s", open_error ? open_error : "missing symbols");
    return r;
}

void nccl_check(ncclResult_t e, const char *what) {
    if (e != ncclSuccess) {
        Rccl &r = rccl();
        bwtmi::fail(BWTMI_E_HIP, "%s failed: %s", what, r.GetErrorString ? r.GetErrorString(e) : "rccl error");
    }
}

}  // namespace

using namespace bwtmi;

struct bwtmi_comm {
    int device = 0, world = 1, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;   // its own stream: never queued behind a context's index build
    DBuf buf;
};

template <class F>
static int cguard(F &&f) {
    try {
        f();
        return BWTMI_OK;
    } catch (const Error &e) {
        set_error("%s", e.msg.c_str());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("out of host memory");
        return BWTMI_E_NOMEM;
    } catch (const std::exception &e) {
        set_error("%s", e.what());
        return BWTMI_E_STATE;
    }
}

extern "C" {

int bwtmi_comm_unique_id(uint8_t *id) {
    return cguard([&] {
        if (!id) fail(BWTMI_E_ARG, "null id");
        ncclUniqueId u;
        nccl_check(rccl().GetUniqueId(&u), "ncclGetUniqueId");
        std::memcpy(id, u.internal, sizeof u.internal);
    });
}

int bwtmi_comm_init(int32_t device, int32_t world, int32_t rank, const uint8_t *id, bwtmi_comm **out) {
    return cguard([&] {
        if (!id || !out || world < 1 || rank < 0 || rank >= world) fail(BWTMI_E_ARG, "bad argument");
        *out = nullptr;
        HIPCHECK(hipSetDevice(device));
        auto *c = new bwtmi_comm();
        c->device = device;
        c->world = world;
        c->rank = rank;
        try {
            HIPCHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
            ncclUniqueId u;
            std::memcpy(u.internal, id, sizeof u.internal);
            nccl_check(rccl().CommInitRank(&c->comm, world, u, rank), "ncclCommInitRank");
            c->buf.ensure(4096);
        } catch (...) {
            if (c->stream) (void)hipStreamDestroy(c->stream);
            delete c;
            throw;
        }
        *out = c;
    });
}

// in-place all-reduce of `count` host values: dtype 0 = int64, 1 = float64; op 0 = sum, 1 = max
int bwtmi_comm_allreduce(bwtmi_comm *c, void *vals, int64_t count, int32_t dtype, int32_t op) {
    return cguard([&] {
        if (!c || (!vals && count) || count < 0 || dtype < 0 || dtype > 1 || op < 0 || op > 1)
            fail(BWTMI_E_ARG, "bad argument");
        if (count == 0) return;
        HIPCHECK(hipSetDevice(c->device));
        const size_t bytes = (size_t)count * 8;
        c->buf.ensure(bytes);
        HIPCHECK(hipMemcpyAsync(c->buf.p, vals, bytes, hipMemcpyHostToDevice, c->stream));
        nccl_check(rccl().AllReduce(c->buf.p, c->buf.p, (size_t)count, dtype == 0 ? ncclInt64 : ncclFloat64,
                                    op == 0 ? ncclSum : ncclMax, c->comm, c->stream),
                   "ncclAllReduce");
        HIPCHECK(hipMemcpyAsync(vals, c->buf.p, bytes, hipMemcpyDeviceToHost, c->stream));
        HIPCHECK(hipStreamSynchronize(c->stream));
    });
}

int bwtmi_comm_free(bwtmi_comm *c) {
    return cguard([&] {
        if (!c) return;
        (void)hipSetDevice(c->device);
        if (c->stream) (void)hipStreamSynchronize(c->stream);
        if (c->comm) (void)rccl().CommDestroy(c->comm);
        c->buf.release();
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
    });
}

// every queued device operation of this process on `device` has finished
int bwtmi_device_sync(int32_t device) {
    return cguard([&] {
        HIPCHECK(hipSetDevice(device));
        HIPCHECK(hipDeviceSynchronize());
    });
}

}  // extern "C"
