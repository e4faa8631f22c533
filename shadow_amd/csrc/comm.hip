// comm.hip — RCCL (dlopen), in-process and modelled collective backends for the routing build.
#include "comm.h"

#include <dlfcn.h>

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
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

using RcclError = CommError;

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
// Several contexts of ONE process (threads), on one GPU (tests) or one per GPU (srg_multi).
// Every collective is two host rendezvous around stream-ordered device work: each rank publishes
// its buffer pointer and an "arrived" event, then every rank PULLS the peers' segments with one
// copy kernel (all peers at once: over xGMI when the devices differ, peer access enabled at
// attach time), records "done", and waits for the peers' "done" before its stream may touch its
// buffer again (a peer may still be reading its segment).
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
        void* xlb = nullptr;         // share_ptrs: line-buffer block, arrival flags, proposed flag value
        uint32_t* xflags = nullptr;
        uint32_t xepoch = 0;
    };
    std::vector<Slot> slots;
    bool aborted = false;  // a rank failed outside the collective protocol: release the others
    explicit LocalGroup(int n_) : n(n_), slots(n_) {}
    void barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) throw RcclError("a peer rank of the in-process group failed");
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || aborted; });
            if (aborted) throw RcclError("a peer rank of the in-process group failed");
        }
    }
};

void local_group_abort(LocalGroup* g) {
    std::lock_guard<std::mutex> lk(g->mu);
    g->aborted = true;
    g->cv.notify_all();
}

void local_group_reset(LocalGroup* g) {
    std::lock_guard<std::mutex> lk(g->mu);
    g->aborted = false;
    g->arrived = 0;
    ++g->gen;
}

namespace {

void hip_ok(hipError_t e, const char* what) {
    if (e != hipSuccess) throw RcclError(std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int kMaxSegs = 32;
struct Segs {
    const unsigned char* src[kMaxSegs];
    unsigned char* dst[kMaxSegs];
    size_t bytes[kMaxSegs];
    unsigned blk0[kMaxSegs + 1];  // first workgroup of each segment
    int n;
};

// one launch copies every segment (peer -> local): workgroups are dealt to segments in
// proportion to their size, 16-B vectors when both ends allow it
__global__ void __launch_bounds__(256) k_pull_segs(Segs s) {
    int q = 0;
    while (q + 1 < s.n && blockIdx.x >= s.blk0[q + 1]) ++q;
    const unsigned nb = s.blk0[q + 1] - s.blk0[q], b = blockIdx.x - s.blk0[q];
    const unsigned char* src = s.src[q];
    unsigned char* dst = s.dst[q];
    const size_t bytes = s.bytes[q];
    const size_t stride = (size_t)nb * blockDim.x, t = (size_t)b * blockDim.x + threadIdx.x;
    size_t done = 0;
    if (((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        const v4u* s16 = reinterpret_cast<const v4u*>(src);
        v4u* d16 = reinterpret_cast<v4u*>(dst);
        const size_t n16 = bytes / 16;
        size_t i = t;
        for (; i + 3 * stride < n16; i += 4 * stride) {
            const v4u x0 = s16[i], x1 = s16[i + stride], x2 = s16[i + 2 * stride], x3 = s16[i + 3 * stride];
            d16[i] = x0;
            d16[i + stride] = x1;
            d16[i + 2 * stride] = x2;
            d16[i + 3 * stride] = x3;
        }
        for (; i < n16; i += stride) d16[i] = s16[i];
        done = n16 * 16;
    }
    for (size_t k = done + t; k < bytes; k += stride) dst[k] = src[k];
}

void launch_pull(std::vector<Segs>& batches, hipStream_t s) {
    for (Segs& sg : batches) {
        if (!sg.n) continue;
        size_t total = 0;
        for (int q = 0; q < sg.n; ++q) total += sg.bytes[q];
        const unsigned budget = 2048;  // workgroups per launch
        unsigned acc = 0;
        for (int q = 0; q < sg.n; ++q) {
            sg.blk0[q] = acc;
            const double share = total ? (double)sg.bytes[q] / (double)total : 0.0;
            acc += std::max(1u, (unsigned)(share * budget));
        }
        sg.blk0[sg.n] = acc;
        k_pull_segs<<<acc, 256, 0, s>>>(sg);
        hip_ok(hipGetLastError(), "k_pull_segs");
    }
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
    void arrive(void* buf, hipStream_t s) {
        auto& me = g->slots[rank];
        me.ptr = buf;
        hip_ok(hipEventRecord(me.ev_arrive, s), "hipEventRecord");
        g->barrier();
    }
    // after the pulls: nobody reuses its buffer until every peer has finished reading it
    void depart(hipStream_t s) {
        hip_ok(hipEventRecord(g->slots[rank].ev_done, s), "hipEventRecord");
        g->barrier();
        for (int p = 0; p < nranks; ++p)
            if (p != rank) hip_ok(hipStreamWaitEvent(s, g->slots[p].ev_done, 0), "hipStreamWaitEvent");
    }
    void bcast(void* buf, size_t bytes, int root, hipStream_t s) override {
        if (nranks == 1 || !bytes) return;
        arrive(buf, s);
        if (rank != root) {
            hip_ok(hipStreamWaitEvent(s, g->slots[root].ev_arrive, 0), "hipStreamWaitEvent");
            std::vector<Segs> b(1);
            b[0].n = 1;
            b[0].src[0] = static_cast<const unsigned char*>(g->slots[root].ptr);
            b[0].dst[0] = static_cast<unsigned char*>(buf);
            b[0].bytes[0] = bytes;
            launch_pull(b, s);
        }
        depart(s);
    }
    void allgatherv(void* buf, const size_t* offs, const size_t* lens, hipStream_t s) override {
        if (nranks == 1) return;
        arrive(buf, s);
        std::vector<Segs> batches;
        for (int p = 0; p < nranks; ++p) {
            if (p == rank || !lens[p]) continue;
            hip_ok(hipStreamWaitEvent(s, g->slots[p].ev_arrive, 0), "hipStreamWaitEvent");
            if (batches.empty() || batches.back().n == kMaxSegs) batches.emplace_back(), batches.back().n = 0;
            Segs& sg = batches.back();
            sg.src[sg.n] = static_cast<const unsigned char*>(g->slots[p].ptr) + offs[p];
            sg.dst[sg.n] = static_cast<unsigned char*>(buf) + offs[p];
            sg.bytes[sg.n] = lens[p];
            ++sg.n;
        }
        launch_pull(batches, s);
        depart(s);
    }
    int device_exchange() const override { return 2; }
    bool distinct_devices() const override {
        std::lock_guard<std::mutex> lk(g->mu);
        for (int p = 0; p < g->n; ++p)
            for (int q = p + 1; q < g->n; ++q)
                if (g->slots[p].device == g->slots[q].device) return false;
        return true;
    }
    void share_ptrs(void* lb, uint32_t* flags, void** lbs, uint32_t** fl, bool* sys, uint32_t* epoch) override {
        g->slots[rank].xlb = lb;
        g->slots[rank].xflags = flags;
        g->slots[rank].xepoch = *epoch;
        g->barrier();
        bool other = false;
        uint32_t ep = 0;
        for (int p = 0; p < nranks; ++p) {
            lbs[p] = g->slots[p].xlb;
            fl[p] = g->slots[p].xflags;
            other |= g->slots[p].device != device;
            ep = std::max(ep, g->slots[p].xepoch);
        }
        *sys = other;
        *epoch = ep;
        g->barrier();  // every rank has read every slot
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
// Timing aid only: rank `rank` of `nranks` runs its share of the schedule alone on one GPU; no
// data moves (results are NOT valid), but every collective costs what the model says it would
// on the MI355X xGMI mesh, as a device-side wait on the stream: latency + the largest per-link
// transfer, links in parallel (allgatherv: each peer's segment arrives over its own link;
// bcast: the root sends over N-1 links at once).  Defaults 15 us and 64 GB/s per link and
// direction; SRG_SIM_COLL_US / SRG_SIM_LINK_GBPS override them (cost model).
__global__ void k_spin_ns(unsigned long long ns) {
    // wall_clock64 ticks at a constant 100 MHz
    const unsigned long long t0 = wall_clock64(), ticks = ns / 10;
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

struct ModelComm final : Comm {
    double lat_ns = 15000.0, gbps = 64.0;
    double flag_ns = 3000.0;  // device-side exchange: a peer's flag over xGMI (SRG_SIM_FLAG_US)
    const char* kind() const override { return "simulated"; }
    int device_exchange() const override { return 1; }
    // the device-side line exchange inside the fused FW launch: every peer's segment arrives over
    // its own link (peers store while they compute, so this is a bound), then its flag
    double model_xchg_ns(size_t max_seg_bytes) const override { return flag_ns + max_seg_bytes / gbps; }
    void wait(double ns, hipStream_t s) {
        if (ns <= 0) return;
        k_spin_ns<<<1, 64, 0, s>>>((unsigned long long)ns);
        hip_ok(hipGetLastError(), "k_spin_ns");
    }
    void bcast(void*, size_t bytes, int, hipStream_t s) override {
        if (nranks > 1 && bytes) wait(lat_ns + bytes / gbps, s);
    }
    void allgatherv(void*, const size_t*, const size_t* lens, hipStream_t s) override {
        if (nranks == 1) return;
        size_t mx = 0;
        for (int p = 0; p < nranks; ++p)
            if (p != rank) mx = std::max(mx, lens[p]);
        wait(lat_ns + mx / gbps, s);
    }
    void allreduce_max_u32(uint32_t*, size_t, hipStream_t s) override {
        if (nranks > 1) wait(lat_ns, s);
    }
};
}  // namespace

Comm* null_create(int nranks, int rank) {
    auto* c = new ModelComm();
    c->nranks = nranks;
    c->rank = rank;
    if (const char* e = std::getenv("SRG_SIM_COLL_US")) c->lat_ns = std::atof(e) * 1e3;
    if (const char* e = std::getenv("SRG_SIM_LINK_GBPS")) c->gbps = std::atof(e);
    if (const char* e = std::getenv("SRG_SIM_FLAG_US")) c->flag_ns = std::atof(e) * 1e3;
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
    // peer access both ways with every rank already attached on another device, so that the
    // pull kernels read peer HBM directly over xGMI (no staging through the host)
    {
        std::lock_guard<std::mutex> lk(g->mu);
        for (int p = 0; p < g->n; ++p) {
            if (p == rank || !g->slots[p].ev_arrive || g->slots[p].device == device) continue;
            const int d2 = g->slots[p].device;
            int ok12 = 0, ok21 = 0;
            if (hipDeviceCanAccessPeer(&ok12, device, d2) != hipSuccess || hipDeviceCanAccessPeer(&ok21, d2, device) != hipSuccess ||
                !ok12 || !ok21)
                return "devices " + std::to_string(device) + " and " + std::to_string(d2) + " cannot access each other's memory";
            for (auto [a, b] : {std::pair<int, int>{device, d2}, std::pair<int, int>{d2, device}}) {
                if (hipSetDevice(a) != hipSuccess) return "hipSetDevice failed";
                const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return "hipDeviceEnablePeerAccess failed";
                (void)hipGetLastError();  // clear a sticky "already enabled"
            }
            if (hipSetDevice(device) != hipSuccess) return "hipSetDevice failed";
        }
    }
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
