// msx_kernels.h — host-side launch interface of the gfx950 combine kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include "msx_types.h"

namespace msx {

// Completion counters of the engine's flag-posting kernels: a transport owns
// kCountBlocks blocks of kCountWords zeroed words (push_counter()): block 0
// word 0 counts k_push_post / the fused push; block 1 is k_push_wait's bulk
// push, block 2 the two-step tree's result count.  Inside a block, word 0 is
// the top level, word 1 a launch count, and kCountSubs sub-counters sit 16
// words (64 B) apart from kCountSubBase (see count_done).
constexpr unsigned kCountSubs = 32;
constexpr unsigned kCountSubBase = 64;
constexpr unsigned kCountWords = 1024;
constexpr unsigned kCountBlocks = 4;

// Launch geometry of the streaming combine.
struct LaunchCfg {
    int variant = 0;      // fp32-SUM tuning variant (0 = default); other pairs ignore it
    int grid_cap = 0;     // 0 = one tile per workgroup (no grid-stride), else max workgroups
    bool host = false;    // launched by the host-memory path of MPI_Reduce_local (zero-copy
                          // over PCIe, or a staged chunk): the k_combine_host symbol, so
                          // profiles keep the device-resident kernel's statistics apart
};

// inout[i] = op(inout[i], in[i]) for i in [0, count), stream-ordered on `s`.
// in / inout must be device-accessible from the current device.
// Returns hipSuccess, or hipErrorInvalidValue for a pair with no kernel.
hipError_t launch_combine(int opidx, Kind k, const void* in, void* inout, size_t count,
                          hipStream_t s, const LaunchCfg& cfg);

// Reference-order tree combine over p inputs (p = 1..8):
//   out[i] = T(srcs[0][i], ..., srcs[p-1][i]) where T is the balanced binary
//   tree of the reference's recursive-halving/doubling schedules with the
//   left operand as `inout`:  ((s0 op s1) op (s2 op s3)) op ((s4 op s5) op ...)
// `srcs` is a device-visible array of p pointers (may be peer pointers).
// `out` may alias srcs[0].
hipError_t launch_tree(int opidx, Kind k, const void* const* srcs_dev, int p, void* out,
                       size_t count, hipStream_t s);

// General schedule-faithful combine (see k_tree in msx_kernels.hip):
//   chain == false: P (power of two <= 16) leaves; leaf i = src[2i] if bit i of
//     pairmask is clear, else src[2i] op src[2i+1] (the non-power-of-two fold);
//     then the balanced tree over the leaves, left operand = inout.
//   chain == true: ((src[0] op src[1]) op src[2]) ... op src[P-1], P <= 16.
struct TreeSpec {
    const void* src[32] = {};
    int P = 1;
    int nleaves = 0;        // 0 = P; else leaves [nleaves, P) are absent (binomial trees)
    unsigned pairmask = 0;
    bool chain = false;
    bool sys = false;   // sources/output shared with peers: system acquire/release
    void* extra[31] = {};   // the result is also stored here (e.g. peers' windows)
    int nextra = 0;
    // GPU-side arrival wait (barrier-free small allreduce): before reading,
    // every workgroup waits until wait_flags[r] >= wait_seq for all r < wait_n,
    // r != wait_skip (flags posted by peers with launch_post_flags); after
    // flag_wait_seconds() without them it stores wait_tag * 65536 + 1 + r (r =
    // the first peer missing) to *wait_err (host-visible) and exits.
    const unsigned long long* wait_flags = nullptr;
    unsigned long long wait_seq = 0;
    int wait_n = 0;
    int wait_skip = -1;
    int* wait_err = nullptr;
    int wait_tag = 1;
    // Fused push (the barrier-free small allreduce in one launch): extra
    // workgroups copy push_n[i] bytes push_src[i] -> push_dst[i] with
    // system-coherent stores and, once all of them completed, store push_seq
    // to every push_flags[j] -- k_push_post's work, in the tree's launch.
    // push_counter: the transport's zeroed completion word (left zero again).
    int push_nseg = 0;
    const void* push_src[32] = {};
    void* push_dst[32] = {};
    size_t push_n[32] = {};
    int push_nflags = 0;
    unsigned long long* push_flags[64] = {};
    unsigned long long push_seq = 0;
    unsigned* push_counter = nullptr;
    bool push_sys = false;
    // Result-ready flags: when the tree workgroups of all `done_launches`
    // launches of one call (this one included; stream-ordered) have stored
    // their results, store done_seq to every done_flags[j] (system scope).
    // done_counter: a zeroed kCountWords block of the transport, left zero again.
    unsigned* done_counter = nullptr;
    unsigned done_launches = 1;
    int done_nflags = 0;
    unsigned long long* done_flags[64] = {};
    unsigned long long done_seq = 0;
};
hipError_t launch_tree_spec(int opidx, Kind k, const TreeSpec& t, void* out, size_t count,
                            hipStream_t s);

// Store `seq` to *dst[i] for i < n (system scope): the arrival flags of the
// barrier-free small allreduce, posted after the data kernel on the same stream.
hipError_t launch_post_flags(unsigned long long* const* dst, int n, unsigned long long seq, hipStream_t s);

// The barrier-free allreduce's push: copy nseg ranges (one grid row each) and,
// once every workgroup's stores are visible system-wide, store `seq` to every
// flags[i] -- one launch, the flag ordered after the data by the kernel itself.
// `counter`: a zeroed device word owned by the caller's transport (the kernel
// leaves it zero again); launches sharing one counter must not overlap.
hipError_t launch_push_post(const void* const* src, void* const* dst, const size_t* nbytes, int nseg,
                            unsigned long long* const* flags, int nflags, unsigned long long seq, bool sys,
                            unsigned* counter, hipStream_t s);

// launch_push_post's push and flags (nseg may be 0: the flags are then
// posted by the waiting workgroup itself), plus ONE workgroup that waits until
// wait_flags[r] >= seq for r < wait_n, r != wait_skip (flag_wait_seconds()
// bound, then wait_tag * 65536 + 1 + r -> *wait_err).  Launches after it on
// `s` read what the flags announce.
hipError_t launch_push_wait(const void* const* src, void* const* dst, const size_t* nbytes, int nseg,
                            unsigned long long* const* flags, int nflags, unsigned long long seq, bool sys,
                            unsigned* counter, const unsigned long long* wait_flags, int wait_n, int wait_skip,
                            int* wait_err, hipStream_t s, int wait_tag = 1);
// Bound of every GPU flag wait: MSX_FLAG_TIMEOUT_MS (default 20000), in
// s_memrealtime ticks and in seconds.
unsigned long long flag_wait_ticks();
double flag_wait_seconds();

// Copy nseg independent byte ranges in one launch (one grid row per segment),
// used to pull allgather blocks from every peer concurrently.
hipError_t launch_copy_segs(const void* const* src, void* const* dst, const size_t* nbytes,
                            int nseg, bool sys, hipStream_t s);

// Tuning of the collective tree combine (fp32 SUM only; other pairs use the
// default): mode 0 = default (loads interleaved with the combines, plain),
// 1 = all sources loaded up front, 2 = up front + non-temporal,
// 3 = interleaved + non-temporal;
// grid_cap 0 = default cap.  Returns 0, or -1 for an invalid setting.
struct TreeTune { int mode = 0; int grid_cap = 0; };
int tree_tune_set(int mode, int grid_cap);
// realigning combine (mutually misaligned operands): 0 = DPP lane shift, 1 = ds_bpermute
int shift_tune_set(int mode);

// HBM ceiling probe (measurement only, see k_probe): mode 0 reads a and b,
// 1 writes b, 2 copies a -> b, 3 reads a; `bytes` per stream, 16-B aligned.
hipError_t launch_probe(int mode, const void* a, void* b, size_t bytes, hipStream_t s);
// pack/unpack geometry: 0 by size, 1 grid-stride form, 2 tile form (msx_pack.hip)
int pack_tune_set(int mode);
// one aligned local copy in a forced geometry: dram = 0 k_copy_segs, 1 k_copy_dram
hipError_t launch_copy_one(const void* src, void* dst, size_t nbytes, hipStream_t s, int dram);

// Number of tuning variants compiled for the fp32 SUM hot path.
int combine_variant_count();
const char* combine_variant_name(int v);

}  // namespace msx
