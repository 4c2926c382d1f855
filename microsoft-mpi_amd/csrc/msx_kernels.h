// msx_kernels.h — host-side launch interface of the gfx950 combine kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include "msx_types.h"

namespace msx {

// Completion counters of the engine's flag-posting kernels: a transport owns
// kCountBlocks blocks of kCountWords zeroed words (push_counter()): block 1 is
// k_push_wait's push, block 2 the two-step tree's result count (block 0 is
// unused).  Inside a block, word 0 is
// the top level, word 1 a launch count, and kCountSubs sub-counters sit 16
// words (64 B) apart from kCountSubBase (see count_done).
constexpr unsigned kCountSubs = 32;
constexpr unsigned kCountSubBase = 64;
constexpr unsigned kCountWords = 1024;
constexpr unsigned kCountBlocks = 4;

// Launch geometry of the streaming combine.
struct LaunchCfg {
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
    void* extra[31] = {};   // the result is also stored here (e.g. peers' windows)
    int nextra = 0;
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

// Store `seq` to *dst[i] for i < n (system scope), in stream order after the
// launches before it (flags that announce no data of their own).
hipError_t launch_post_flags(unsigned long long* const* dst, int n, unsigned long long seq, hipStream_t s);

// The GPU-flag schedules' synchronisation point, one launch: copy nseg ranges
// (each below 4 GiB) into peer windows with write-through stores and, once
// every workgroup's stores completed, store `seq` to every flags[i] (nseg may
// be 0: the flags are then posted by the waiting workgroup itself); plus ONE
// workgroup that waits until wait_flags[r] >= seq for r < wait_n, r !=
// wait_skip (flag_wait_seconds() bound, then wait_tag * 65536 + 1 + r ->
// *wait_err).  Launches after it on `s` read what the flags announce.
// `counter`: a zeroed kCountWords block of the caller's transport (left zero
// again); launches sharing one counter must not overlap.
hipError_t launch_push_wait(const void* const* src, void* const* dst, const size_t* nbytes, int nseg,
                            unsigned long long* const* flags, int nflags, unsigned long long seq,
                            unsigned* counter, const unsigned long long* wait_flags, int wait_n, int wait_skip,
                            int* wait_err, hipStream_t s, int wait_tag = 1);
// Bound of every GPU flag wait: MSX_FLAG_TIMEOUT_MS (default 20000), in
// s_memrealtime ticks and in seconds.
unsigned long long flag_wait_ticks();
double flag_wait_seconds();

// Copy nseg independent byte ranges in one launch (one grid row per segment),
// used to pull allgather blocks from every peer concurrently.
hipError_t launch_copy_segs(const void* const* src, void* const* dst, const size_t* nbytes,
                            int nseg, hipStream_t s);

// pack/unpack geometry (test hook, msx_tune_pack): 0 by size, 1 grid-stride
// form, 2 tile form (msx_pack.hip); the accumulate always runs its tile form
int pack_tune_set(int mode);

}  // namespace msx
