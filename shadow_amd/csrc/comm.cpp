// comm.cpp — RCCL (dlopen) and in-process collective backends for the routing build.
#include "comm.h"

#include <dlfcn.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <stdexcept>
#include <vector>

namespace srg {

namespace {

// ---- RCCL, resolved at run time -------------------------------------------------------
// torch ships its own librccl (soname librccl.so.1); when torch is already loaded, dlopen of
// the soname returns that copy, so one RCCL serves both.  Plain C callers get /opt/rocm's.
struct RcclApi {
    bool ok = false;
    std::string err;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (h) break;
        }
        if (!h) {
            api.err = std::string("cannot load librccl: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](auto& fp, const char* name) {
            fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
            if (!fp) all = false;
        };
        sym(api.GetUniqueId, "ncclGetUniqueId");
        sym(api.CommInitRank, "ncclCommInitRank");
        sym(api.CommDestroy, "ncclCommDestroy");
        sym(api.Broadcast, "ncclBroadcast");
        sym(api.AllReduce, "ncclAllReduce");
        sym(api.Send, "ncclSend");
        sym(api.Recv, "ncclRecv");
        sym(api.GroupStart, "ncclGroupStart");
        sym(api.GroupEnd, "ncclGroupEnd");
        sym(api.GetErrorString, "ncclGetErrorString");
        if (!all) {
            api.err = "librccl lacks a required symbol";
            return;
        }
        api.ok = true;
    });
    return api;
}

struct RcclError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

void nccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw RcclError(std::string(what) + ": " + rccl().GetErrorString(r));
}

struct RcclComm final : Comm {
    ncclComm_t comm = nullptr;
    const char* kind() const override { return "rccl"; }
    ~RcclComm() override {
        if (comm) rccl().CommDestroy(comm);
    }
    void bcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (nranks == 1 || !bytes) return;
        nccl_check(rccl().Broadcast(buf, buf, bytes, ncclUint8, root, comm, s), "ncclBroadcast");
    }
    void allgatherv(void* buf, const size_t* offs, const size_t* lens, hipStream_t s) override {
        if (nranks == 1) return;
        // direct point-to-point over the xGMI mesh: my segment to every peer, theirs to me
        auto* b = static_cast<unsigned char*>(buf);
        nccl_check(rccl().GroupStart(), "ncclGroupStart");
        for (int p = 0; p < nranks; ++p) {
            if (p == rank) continue;
            if (lens[rank]) nccl_check(rccl().Send(b + offs[rank], lens[rank], ncclUint8, p, comm, s), "ncclSend");
            if (lens[p]) nccl_check(rccl().Recv(b + offs[p], lens[p], ncclUint8, p, comm, s), "ncclRecv");
        }
        nccl_check(rccl().GroupEnd(), "ncclGroupEnd");
    }
    void allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t s) override {
        if (nranks == 1 || !count) return;
        nccl_check(rccl().AllReduce(buf, buf, count, ncclUint32, ncclMax, comm, s), "ncclAllReduce");
    }
};

}  // namespace

std::string rccl_unique_id(unsigned char out[128]) {
    RcclApi& a = rccl();
    if (!a.ok) return a.err;
    ncclUniqueId id;
    ncclResult_t r = a.GetUniqueId(&id);
    if (r != ncclSuccess) return std::string("ncclGetUniqueId: ") + a.GetErrorString(r);
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    std::memcpy(out, &id, 128);
    return "";
}

std::string rccl_create(int nranks, int rank, const unsigned char id[128], int device, Comm** out) {
    RcclApi& a = rccl();
    if (!a.ok) return a.err;
    if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    auto* c = new RcclComm();
    c->rank = rank;
    c->nranks = nranks;
    ncclResult_t r = a.CommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        c->comm = nullptr;
        delete c;
        return std::string("ncclCommInitRank: ") + a.GetErrorString(r);
    }
    *out = c;
    return "";
}

// ---- in-process group ------------------------------------------------------------------
struct LocalGroup {
    int n;
    std::atomic<int> refs{1};
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    struct Slot {
        void* ptr = nullptr;
        int device = 0;
        hipEvent_t ev_arrive = nullptr, ev_done = nullptr;
        std::vector<uint32_t> host;  // allreduce staging
    };
    std::vector<Slot> slots;
    explicit LocalGroup(int n_) : n(n_), slots(n_) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw RcclError(std::string(what) + ": " + hipGetErrorString(e));
}

struct LocalComm final : Comm {
    LocalGroup* g;
    int device;
    const char* kind() const override { return "local"; }
    ~LocalComm() override {
        auto& sl = g->slots[rank];
        if (sl.ev_arrive) (void)hipEventDestroy(sl.ev_arrive);
        if (sl.ev_done) (void)hipEventDestroy(sl.ev_done);
        sl.ev_arrive = sl.ev_done = nullptr;
        local_group_release(g);
    }
    void copy(void* dst, int dst_dev, const void* src, size_t bytes, hipStream_t s) {
        if (dst_dev == device) hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s), "hipMemcpyAsync");
        else hip_ok(hipMemcpyPeerAsync(dst, dst_dev, src, device, bytes, s), "hipMemcpyPeerAsync");
    }
    void arrive(void* buf, hipStream_t s) {
        auto& me = g->slots[rank];
        me.ptr = buf;
        hip_ok(hipEventRecord(me.ev_arrive, s), "hipEventRecord");
        g->barrier();
    }
    void bcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (nranks == 1 || !bytes) return;
        arrive(buf, s);
        if (rank == root) {
            for (int p = 0; p < nranks; ++p)
                if (p != root) hip_ok(hipStreamWaitEvent(s, g->slots[p].ev_arrive, 0), "hipStreamWaitEvent");
            for (int p = 0; p < nranks; ++p)
                if (p != root) copy(g->slots[p].ptr, g->slots[p].device, buf, bytes, s);
            hip_ok(hipEventRecord(g->slots[root].ev_done, s), "hipEventRecord");
        }
        g->barrier();
        if (rank != root) hip_ok(hipStreamWaitEvent(s, g->slots[root].ev_done, 0), "hipStreamWaitEvent");
    }
    void allgatherv(void* buf, const size_t* offs, const size_t* lens, hipStream_t s) override {
        if (nranks == 1) return;
        arrive(buf, s);
        for (int p = 0; p < nranks; ++p)
            if (p != rank) hip_ok(hipStreamWaitEvent(s, g->slots[p].ev_arrive, 0), "hipStreamWaitEvent");
        auto* b = static_cast<unsigned char*>(buf);
        for (int p = 0; p < nranks; ++p)
            if (p != rank && lens[rank])
                copy(static_cast<unsigned char*>(g->slots[p].ptr) + offs[rank], g->slots[p].device, b + offs[rank],
                     lens[rank], s);
        hip_ok(hipEventRecord(g->slots[rank].ev_done, s), "hipEventRecord");
        g->barrier();
        for (int p = 0; p < nranks; ++p)
            if (p != rank) hip_ok(hipStreamWaitEvent(s, g->slots[p].ev_done, 0), "hipStreamWaitEvent");
    }
    void allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t s) override {
        if (nranks == 1 || !count) return;
        auto& me = g->slots[rank];
        me.host.resize(count);
        hip_ok(hipMemcpyAsync(me.host.data(), buf, count * 4, hipMemcpyDeviceToHost, s), "hipMemcpyAsync");
        hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
        g->barrier();
        std::vector<uint32_t> r(count, 0);
        for (int p = 0; p < nranks; ++p)
            for (size_t i = 0; i < count; ++i) r[i] = std::max(r[i], g->slots[p].host[i]);
        g->barrier();  // everyone has read every slot before anyone reuses its staging
        hip_ok(hipMemcpyAsync(buf, r.data(), count * 4, hipMemcpyHostToDevice, s), "hipMemcpyAsync");
        hip_ok(hipStreamSynchronize(s), "hipStreamSynchronize");
    }
};

}  // namespace

namespace {
// Timing aid only: rank `rank` of `nranks` runs its share of the schedule with every
// collective elided (results are NOT valid).  Used to profile one rank's compute and the FW
// critical path on a single GPU.
struct NullComm final : Comm {
    const char* kind() const override { return "simulated"; }
    void bcast(void*, size_t, int, hipStream_t) override {}
    void allgatherv(void*, const size_t*, const size_t*, hipStream_t) override {}
    void allreduce_max_u32(uint32_t*, size_t, hipStream_t) override {}
};
}  // namespace

Comm* null_create(int nranks, int rank) {
    auto* c = new NullComm();
    c->nranks = nranks;
    c->rank = rank;
    return c;
}

LocalGroup* local_group_create(int nranks) { return new LocalGroup(nranks); }

void local_group_release(LocalGroup* g) {
    if (g && g->refs.fetch_sub(1) == 1) delete g;
}

std::string local_create(LocalGroup* g, int rank, int device, Comm** out) {
    if (!g || rank < 0 || rank >= g->n) return "bad local group rank";
    auto& sl = g->slots[rank];
    if (sl.ev_arrive) return "local group rank already attached";
    if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
    if (hipEventCreateWithFlags(&sl.ev_arrive, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming) != hipSuccess)
        return "hipEventCreate failed";
    sl.device = device;
    g->refs.fetch_add(1);
    auto* c = new LocalComm();
    c->g = g;
    c->device = device;
    c->rank = rank;
    c->nranks = g->n;
    *out = c;
    return "";
}

}  // namespace srg
