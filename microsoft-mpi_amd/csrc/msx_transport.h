// msx_transport.h — multi-rank bootstrap, peer mapping and the collective engine.
//
// One process per GPU on one node.  Ranks find each other through a small TCP
// hub (rank 0 listens on MASTER_ADDR:MSX_BOOTSTRAP_PORT), exchange HIP IPC
// handles of the buffers a collective touches, and then every rank reads its
// peers' HBM directly (xGMI on 8 x MI355X; same-HBM when several ranks share
// one GPU).  The combine runs as one schedule-faithful multi-input kernel, so
// each element sees exactly the association and inout/in roles of the
// reference's recursive-halving / recursive-doubling / pairwise schedules.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <functional>
#include <future>
#include <vector>

#include "msx_comm.h"
#include "msx_dtype.h"

namespace msx {

class Transport {
public:
    virtual ~Transport() = default;
    int rank = 0;
    int size = 1;
    // Single-chunk recursive-doubling calls skip their closing barrier and
    // alternate between two halves of the IN sub-slots (rd_parity); a later
    // window user of another kind barriers first while window_open is set.
    // Every rank runs the same collective sequence, so these agree everywhere.
    bool window_open = false;
    int rd_parity = 0;
    // barrier-free allreduce: sequence number of the last flag-synchronised
    // call (the same on every rank: collectives are called in one order)
    unsigned long long rd_seq = 0;
    // The barrier-free two-step allreduce writes the peers' OUT areas (upper
    // halves); a host-barrier collective may still be reading its own OUT
    // area after its last barrier, so the first two-step call after one
    // barriers first.  Cleared by every host-barrier window user.
    bool out_quiet = false;
    // Whether two or more ranks of this communicator run on one GPU (their
    // PCI bus ids, allgathered at init, so every rank holds the same value).
    // The GPU-flag Rabenseifner schedules default off there (two_step_max).
    bool gpu_shared = false;
    // The engine's second stream belongs to the communicator, so collectives
    // of two communicators running at once from different threads never
    // wait on each other (msx_transport.cpp, aux_stream).
    hipStream_t aux = nullptr;
    // lock-step host collectives over the bootstrap hub (all ranks, same n)
    virtual int allgather(const void* mine, size_t n, void* all) = 0;
    virtual int barrier() = 0;
    // Completion words of the barrier-free small calls (node shared memory):
    // post_done(s) = this rank finished call s; wait_done(r, s) waits for rank r.
    virtual bool has_done() const { return false; }
    virtual void post_done(uint64_t) {}
    virtual int wait_done(int, uint64_t) { return MPI_ERR_OTHER; }
    // Device pointers through which THIS process reads rank r's `ptr`
    // (ptr must be device memory of the calling rank).  Collective.
    virtual int map_peers(const void* ptr, std::vector<char*>& out) = 0;
    // Per-rank device scratch, IPC-mapped once: out[r] = rank r's window.
    virtual int window(size_t bytes, std::vector<char*>& out) = 0;
    // Passive-target staging: a second per-rank window, created by the first
    // call (collective) and kept for the transport's lifetime.  Its size is
    // agreed by all ranks (the minimum of their rma_bytes_for(ranks sharing
    // their GPU)) and returned in *bytes, so every rank addresses the same
    // slots in every peer's area.
    virtual int rma_window(std::vector<char*>& out, size_t* bytes) = 0;
    virtual hipStream_t stream() = 0;
    // Completion counters of the fused push (k_push_post, word 0) and of the
    // two-step allreduce's result flags (words 1-2): zeroed device words per
    // transport, used only by launches on stream(), which the transport
    // issues one collective at a time.  nullptr if allocation failed.
    virtual unsigned* push_counter() = 0;
    // chunks sent to / received from each peer over the windows (the
    // intercommunicator point-to-point channel; both sides count alike)
    uint64_t& p2p_sent(int peer)
    {
        if (p2p_sent_.size() < (size_t)size) p2p_sent_.resize((size_t)size, 0);
        return p2p_sent_[(size_t)peer];
    }
    uint64_t& p2p_recv(int peer)
    {
        if (p2p_recv_.size() < (size_t)size) p2p_recv_.resize((size_t)size, 0);
        return p2p_recv_[(size_t)peer];
    }

private:
    std::vector<uint64_t> p2p_sent_, p2p_recv_;
};

int transport_create(int rank, int size, Transport** out);
// MPI_Comm_split over `parent` (collective): this rank's place in its color's
// group and, for groups of two or more, the group's own transport (hub,
// shared-memory barrier, engine windows).  color MPI_UNDEFINED: no group.
int transport_split(Transport* parent, int color, int key, int* new_rank, int* new_size, Transport** out,
                    std::vector<int>* members = nullptr);   // parent ranks, by new rank
// window-allreduce phase timers (seconds): stage+scatter, collect wait+barrier A,
// reduce+push, barrier B, last collect, chunks, calls; returns 7
int engine_stats(double* out, int n, int reset);
// all-peer remote-write bandwidth probe (collective over c)
int engine_peer_write_probe(Comm* c, size_t bytes, int reps, double* seconds, int64_t* used);
// data plane the engine uses for `tp`: "rccl", "ipc" or "self" (size 1)
const char* engine_transport_name(Transport* tp);
void transport_destroy(Transport* t);

// ---- schedules (pure functions; exported for host-side tests) ----------------
// Reference algorithm selected for an allreduce (reduce.cpp:3884-3888) and for a
// reduce_scatter (reduce.cpp:1705-1750).
enum Algo { A_RECURSIVE_DOUBLING = 0, A_RABENSEIFNER = 1, A_RS_HALVING = 2, A_RS_PAIRWISE = 3,
            A_BINOMIAL = 4 };

struct Leaf { int a = -1, b = -1; };   // real ranks: value = a, or a op b when b >= 0

int pof2_floor(int p);
int newrank_of(int rank, int p);                  // -1 for folded (even, < 2*rem) ranks
int real_of_newrank(int n, int p);
Leaf leaf_of(int n, int p);                       // leaf value of newrank n
int allreduce_algo(int p, size_t count, int type_size, bool builtin);
int reduce_scatter_algo(int p, size_t total_count, int type_size, bool commutative);
// MPI_Reduce (reduce.cpp:151-153): Rabenseifner or binomial
int reduce_algo(int p, size_t count, int type_size, bool builtin);
// allreduce Rabenseifner blocks: block j = [start, start+len), computed at newrank owner
void allreduce_block(int p, size_t count, int j, size_t* start, size_t* len);
// the pipelined two-step allreduce's chunk plan (msx_transport.cpp)
struct TwoStepRange { size_t e0, e1; int owner; };
size_t two_step_chunk_el(int p, size_t esz);
void two_step_plan(int p, size_t count, size_t pc_el, size_t ci, int me, std::vector<TwoStepRange>* ranges,
                   size_t* plo, size_t* phi, size_t* len);
int allreduce_block_owner(int p, int j);           // newrank that owns block j
int allreduce_block_of_newrank(int p, int n);
// Tree spec (in real ranks) for the value newrank n computes:
//   allreduce:      leaves y_k = leaf(n ^ k)
//   reduce_scatter: leaves y_k = leaf(n ^ bitrev(k))   (recursive halving)
//   pairwise:       chain x_r, x_{r-1}, ..., x_{r-p+1}
struct RankTree {
    int P = 1;
    int nleaves = 0;        // 0 = P (binomial trees over non-power-of-two p use fewer)
    unsigned pairmask = 0;
    bool chain = false;
    int src[32];            // real ranks in kernel slot order
};
RankTree tree_allreduce(int p, int n);
RankTree tree_reduce_scatter(int p, int n);
RankTree tree_pairwise(int p, int r);
//   reduce, Rabenseifner: leaves y_k = leafR(n ^ k), leafR = even-first fold
RankTree tree_reduce_rsag(int p, int n);
//   MPI_Ireduce, Rabenseifner: tree_reduce_rsag over root-relative ranks
RankTree tree_ireduce_rsag(int p, int n, int root);
//   reduce, binomial:     leaves x_{(k + root) % p}, k < p, of a nextpow2(p) tree
RankTree tree_reduce_binomial(int p, int root);
// Bytes per element the algorithm gates multiply the count by: the blocking
// calls use MPI_Type_size (reduce.cpp:151, :1705, :3821), the NBC task lists
// of MPI_Iallreduce / MPI_Ireduce the extent (:4712-4717, :6695-6701; 16 vs
// 12 for MPI_DOUBLE_INT, 8 vs 6 for MPI_SHORT_INT); MPI_Ireduce_scatter uses
// the size again (:3201).
int gate_type_size(MPI_Datatype dt, bool nbc);

// ---- engine entry points (msx_comm.cpp routes size > 1 here) ---------------
// nbc: the schedule of the reference's NBC task list (MPI_Iallreduce /
// MPI_Ireduce, or a blocking call under MSMPI_FORCE_ASYNC_WORKFLOW): the
// extent gate and, for MPI_Ireduce's Rabenseifner, root-relative ranks.
int engine_allreduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                     const OpRef& op, bool nbc = false);
int engine_reduce(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                  const OpRef& op, int root, bool nbc = false);
int engine_reduce_scatter(Comm* c, const void* sendbuf, void* recvbuf, const int* recvcounts,
                          MPI_Datatype dt, const OpRef& op);
int engine_scan(Comm* c, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                const OpRef& op, bool exclusive);
// ---- one-sided accumulate (MPI_Win, fence synchronisation) -------------------
// Reference: mpid/win.cpp (MPID_Win_queue, MPIDI_Win_local_accumulate
// :1405-1450) and the target-side apply of mpid/packethandling.cpp
// (do_accumulate_op :2917-3000): remote operations are queued at the origin
// and applied by the TARGET, `target = target op origin` through the op table.
enum RmaKind : int32_t { RMA_PUT = 0, RMA_GET = 1, RMA_ACC = 2, RMA_GACC = 3, RMA_CAS = 4 };
struct RmaDesc {                 // exchanged at synchronisation (plain data)
    int32_t kind = -1;
    int32_t target = -1;
    int32_t opidx = 0;           // builtin op index (O_REPLACE / O_NOOP allowed)
    int32_t dt = 0;              // target MPI_Datatype (its element type when derived)
    int64_t count = 0;           // units: elements, or target-type instances when derived
    int64_t tdisp = 0;           // byte offset in the target's window
    // Derived target datatype (layout >= 0): the target rebuilds it from the
    // origin's serialized runs at int64 offset `layout` of the origin's blob
    // (the reference ships the dataloop the same way, packethandling.cpp).
    int32_t layout = -1;
    int32_t pad_ = 0;
    int64_t usize = 0;           // packed bytes per unit (payload / fetch stride)
    int64_t uext = 0;            // target bytes per unit (extent)
    int64_t span_lo = 0, span_hi = 0;   // target bytes touched, relative to tdisp
};
struct RmaLocal {                // origin-side addresses of a queued operation
    const void* origin = nullptr;   // packed payload (the user's buffer, or tmp_origin)
    void* result = nullptr;         // packed destination of fetched bytes (user's, or tmp_result)
    const void* compare = nullptr;
    void* tmp_origin = nullptr;     // device copy of a derived origin, packed at issue
    void* tmp_result = nullptr;     // device staging of a derived result, unpacked at completion
    void* result_user = nullptr;
    MPI_Datatype result_dt = 0;
    int64_t result_count = 0;
};
struct PassiveState;             // passive-target machinery of one window (engine side)
struct RmaWin {
    int handle = 0;
    Comm* comm = nullptr;
    char* base = nullptr;
    int64_t size = 0;
    int disp_unit = 1;
    std::vector<int64_t> sizes;  // every rank's window size in bytes
    std::vector<int> disp_units; // every rank's disp_unit
    MPI_Errhandler errhandler = MPI_ERRHANDLER_NULL;   // unset: MPI_COMM_WORLD's handler
    std::vector<RmaDesc> q;      // queued remote operations, issue order
    std::vector<RmaLocal> ql;
    std::vector<int64_t> blob;   // serialized derived target layouts of the queued operations
    // passive target (MPI_Win_lock ... MPI_Win_unlock): per target, the lock
    // type of the open access epoch (0 = none) and whether it is acquired yet
    // (remote locks are acquired lazily, at the first flush / unlock, like the
    // reference's queued lock request, win.cpp:1018-1060)
    std::vector<int> lock_mode;
    std::vector<char> lock_held;
    bool lock_all = false;
    PassiveState* passive = nullptr;
    void* owned = nullptr;       // MPI_Win_allocate: memory freed with the window
    // post-start-complete-wait (generalized active target): window ranks of the
    // open access epoch's targets / exposure epoch's origins, and per rank the
    // number of epochs opened so far (matched against the peers' counters)
    bool access_epoch = false;
    int access_assert = 0;
    std::vector<int> access_targets;
    std::vector<uint32_t> starts;     // per target: access epochs opened to it
    bool exposure_epoch = false;
    std::vector<int> exposure_origins;
    std::vector<uint32_t> posts;      // per origin: exposure epochs opened to it
};
// Finish an operation's origin side: unpack a derived result, free temporaries.
int rma_local_complete(RmaLocal& l);
// Apply one operation on this rank's own window memory now (target == self,
// as the reference does, win.cpp:1570-1590); blocking.
int rma_apply_self(RmaWin* w, const RmaDesc& d, const RmaLocal& l, const Dtype* T);
// MPI_Win_fence: every queued operation of every origin is applied at its
// target in (origin rank, issue) order; fetched values are delivered.  Collective.
int engine_rma_fence(RmaWin* w);
int engine_rma_create(RmaWin* w);    // exchange window sizes (collective)
int engine_rma_free(RmaWin* w);      // stop the passive-target service (collective)
// Passive target.  Operations of a lock epoch are queued at the origin; a
// flush / unlock acquires the target's lock (a reader-writer word in shared
// memory), ships each operation's payload into the target's engine window and
// a request into the window's shared-memory mailbox, and waits: the TARGET's
// service thread applies it to its window memory with the op kernels on its
// own GPU (the target-side apply of packethandling.cpp:2917-3060, made
// independent of the target's MPI calls) and returns fetched bytes into the
// origin's window.  One service thread per window serialises all origins, so
// concurrent accumulates under shared locks are element-wise atomic.
int engine_rma_lock(RmaWin* w, int target, int mode);      // blocking acquire
int engine_rma_unlock_target(RmaWin* w, int target);       // release
int engine_rma_flush(RmaWin* w, int target);               // complete queued ops to target
// serialises a self-target apply with the window's service thread
void engine_rma_self_guard(RmaWin* w, bool enter);
// PSCW (mpid/win.cpp:3689-4088).  Post: tell each origin of the group that the
// window is exposed to it (a counter per (target, origin) in the window's
// shared memory).  Complete: for each target of the start group, wait for its
// post (unless MPI_MODE_NOCHECK), ship the queued operations (applied by the
// target's service thread, as a flush), then count this origin's epoch done at
// the target.  Wait / test: every origin of the posted group counted done.
int engine_rma_post(RmaWin* w);
int engine_rma_complete(RmaWin* w);
int engine_rma_wait(RmaWin* w, bool block, int* flag);

// Run `fn` on the collective worker thread, after every collective issued
// before it (MPI issue order); re-entrant calls from the worker run inline.
std::shared_future<int> engine_async(std::function<int()> fn);

// MPI_Comm_split / MPI_Comm_dup (collective over `parent`, in issue order with
// its collectives): *out = the new communicator, or nullptr for
// MPI_COMM_NULL (color MPI_UNDEFINED).  The handle is assigned by the caller.
int engine_comm_split(Comm* parent, int color, int key, Comm** out);
// World shared-memory mailbox (collective at MPI_Init, p > 1): small host
// messages between any two processes, matched by (source process, tag).
int engine_mailbox_init(Transport* world, int rank, int size);
// MPI_Intercomm_create over `local` (collective over both groups); the
// leaders exchange their groups through the mailbox.  `peer` / `remote_leader`
// are significant at the local leader only.
int engine_intercomm_create(Comm* local, int local_leader, Comm* peer, int remote_leader, int tag, Comm** out);
int engine_intercomm_merge(Comm* inter, int high, Comm** out);
int engine_intercomm_dup(Comm* inter, Comm** out);
// Intercommunicator reductions (reduce.cpp:778-863, 1821-1990, 4109-4175):
// root = MPI_ROOT / MPI_PROC_NULL / a remote rank as MPI_Reduce defines them.
int engine_inter_reduce(Comm* ic, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                        const OpRef& op, int root);
int engine_inter_allreduce(Comm* ic, const void* sendbuf, void* recvbuf, size_t count, MPI_Datatype dt,
                           const OpRef& op);
int engine_inter_reduce_scatter(Comm* ic, const void* sendbuf, void* recvbuf, const int* recvcounts,
                                MPI_Datatype dt, const OpRef& op);
// MPI_Comm_free (collective): tears down the communicator's transport.
int engine_comm_free(Comm* c);

}  // namespace msx
