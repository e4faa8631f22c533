// comm.h — collectives used by the multi-GPU routing build.
//
// The reference has no communication at all (rayon threads in one process, mod.rs:190-208);
// these are the exchange steps of the MI355X design:
//   bcast      FW pivot row panel, in place, root = owner of the pivot block
//   allgatherv row-block segments (essential-edge bitmask, output rows): every rank holds the
//              same layout and contributes [offs[rank], offs[rank] + lens[rank]) bytes
//   allreduce_max_u32  small flags (u32 certification, unreachable pairs)
// All calls are stream-ordered: they start when `s` reaches them and later work on `s` sees
// the result, like RCCL.  Every rank issues the same sequence of calls.
//
// Backends: RCCL over xGMI (one process per GPU, librccl loaded with dlopen on first use), and
// an in-process group (several contexts in one process, e.g. several ranks on one GPU) used to
// test the distributed schedule bit-exactly where only one GPU is available.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace srg {

// a collective failed (RCCL error, or a peer rank of an in-process group failed): SRG_ERR_RCCL
struct CommError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct Comm {
    int rank = 0, nranks = 1;
    virtual ~Comm() = default;
    virtual const char* kind() const = 0;
    virtual void bcast(void* buf, size_t bytes, int root, hipStream_t s) = 0;
    virtual void allgatherv(void* buf, const size_t* offs, const size_t* lens, hipStream_t s) = 0;
    virtual void allreduce_max_u32(uint32_t* buf, size_t count, hipStream_t s) = 0;
    // Device-side exchange of the FW line buffers (xchg.hip.h k_line_xchg): 0 = not available
    // (collectives only), 1 = modelled (a simulated rank: the exchange waits model_xchg_ns), 2 = peer
    // pointers (share_ptrs).
    virtual int device_exchange() const { return 0; }
    virtual double model_xchg_ns(size_t) const { return 0.0; }
    // every rank on its own device
    virtual bool distinct_devices() const { return false; }
    // collective: every rank publishes its line-buffer block and arrival-flag array and proposes the
    // build's flag value; on return lbs[r] / flags[r] are rank r's (reachable from this rank's
    // kernels), sys = some rank is on another device (system-scope fences and stores), *epoch = the
    // largest value proposed (every rank raises and waits for the same value)
    virtual void share_ptrs(void*, uint32_t*, void** lbs, uint32_t** flags, bool* sys, uint32_t* epoch) {
        (void)lbs, (void)flags, (void)sys, (void)epoch;
        throw CommError("device-side exchange unsupported by this communicator");
    }
};

// RCCL: unique id (128 bytes) from rank 0, shared by the caller, then init on every rank.
// Return "" on success, else an error message.
std::string rccl_unique_id(unsigned char out[128]);
std::string rccl_create(int nranks, int rank, const unsigned char id[128], int device, Comm** out);

// Timing aid: collectives move nothing (results invalid) but cost the modelled xGMI time on the
// stream, see SRG_OPT_SIMULATE_RANK and DESIGN.md §7.
Comm* null_create(int nranks, int rank);

// In-process group of `nranks` ranks (threads of one process); each rank attaches one context.
struct LocalGroup;
LocalGroup* local_group_create(int nranks);
void local_group_release(LocalGroup* g);  // refcounted: the group and each attached comm
std::string local_create(LocalGroup* g, int rank, int device, Comm** out);
// a rank failed outside the collective protocol: every barrier of the group throws until reset
void local_group_abort(LocalGroup* g);
void local_group_reset(LocalGroup* g);

}  // namespace srg
