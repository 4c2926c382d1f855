// msx_tree_dev.h — device code shared by msx_kernels.hip (push / flag / copy
// kernels) and the msx_tree_*.hip parts (the reference-order tree combine
// k_tree, instantiated per MPI_Op in separate translation units so they
// compile in parallel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "msx_dev_ops.h"
#include "msx_kernels.h"

namespace msx {
namespace dev {

// ---- copy-segment and flag descriptors (k_copy_segs, k_push_wait, k_tree) -------
constexpr int kMaxSegs = 32;
struct CopySegs {
    const void* src[kMaxSegs];
    void* dst[kMaxSegs];
    size_t nbytes[kMaxSegs];
    int n;
};

struct PostFlags {
    unsigned long long* dst[64];
    unsigned long long seq;
    int n;
};

// "This lane's stores have completed" without a cache maintenance operation:
// s_waitcnt vmcnt(0) (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15).  An
// agent-scope release fence would do the same wait but also write back the
// whole XCD L2 (buffer_wbl2), once per workgroup -- on this multi-XCD part
// that made a 2048-workgroup push 20x slower.  Window memory is uncached
// (MTYPE_UC), so a completed store is at the owner; nothing sits in L2.
__device__ __forceinline__ void stores_done()
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);      // no compiler motion of stores past the wait
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Write-through stores for data a GPU flag announces to another GPU: relaxed
// system-scope atomic stores, i.e. global_store_* sc0 sc1, which the L2 passes
// through to the owner's memory whatever MTYPE the importer maps the peer
// window with.  Once such a store has completed (stores_done), it is visible
// at the owner, so the flag protocol does not rest on the windows being
// mapped uncached on the WRITER (an NC mapping would leave plain stores dirty
// in this XCD's L2, where only an L2 writeback, ~20x slower per workgroup,
// could push them out).
__device__ __forceinline__ void st_wt(u32x4* p, u32x4 v)
{
    unsigned long long* d = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(d, (unsigned long long)v.x | ((unsigned long long)v.y << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(d + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
}

// 16-byte write-through stores in bulk: buffer_store_dwordx4 with the same
// sc0 sc1 policy (aux 17), through a raw buffer resource on a workgroup-
// uniform base (wt_rsrc) and a byte offset below 4 GiB (the launchers only
// set `wt` for ranges that satisfy this).  Half the store instructions of
// st_wt's two 8-byte atomics.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(void* base)
{
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)0xFFFFFFFF, 0x00020000);
}
__device__ __forceinline__ void st_wt_at(__amdgpu_buffer_rsrc_t r, size_t off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)(unsigned)off, 0, 17);
}

// One element of 1, 2, 4, 8 or 16 bytes, write-through (the scalar tails).
template <class T>
__device__ __forceinline__ void st_wt_elem(T* p, const T& v)
{
    static_assert(sizeof(T) == 1 || sizeof(T) == 2 || sizeof(T) == 4 || sizeof(T) == 8 || sizeof(T) == 16,
                  "element size");
    if constexpr (sizeof(T) == 16) {
        u32x4 w;
        __builtin_memcpy(&w, &v, 16);
        st_wt(reinterpret_cast<u32x4*>(p), w);
    } else {
        using W = typename std::conditional<sizeof(T) == 1, unsigned char,
                  typename std::conditional<sizeof(T) == 2, unsigned short,
                  typename std::conditional<sizeof(T) == 4, unsigned, unsigned long long>::type>::type>::type;
        W w;
        __builtin_memcpy(&w, &v, sizeof(T));
        __hip_atomic_store(reinterpret_cast<W*>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Count finished workgroup b of nb; true in exactly one workgroup, after all
// nb have counted.  Thousands of workgroups adding to ONE word serialise
// (a 4096-workgroup tree took 70 us instead of 38), so workgroup b counts on
// sub-counter b % kCountSubs (its own 64-byte line, base[kCountSubBase +
// 16 i]) and only the last of each sub-counter counts on base[0].  Relaxed:
// each add is issued after the workgroup's stores completed (stores_done),
// so when the last add is seen, all of them have.  Words are left zero.
__device__ __forceinline__ bool count_done(unsigned* base, unsigned b, unsigned nb)
{
    const unsigned i = b % kCountSubs;
    const unsigned nsub = nb < kCountSubs ? nb : kCountSubs;
    const unsigned want = (nb - i + kCountSubs - 1) / kCountSubs;   // workgroups on sub-counter i
    unsigned* c = base + kCountSubBase + 16 * i;
    if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != want - 1) return false;
    __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(base, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != nsub - 1) return false;
    __hip_atomic_store(base, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// The push of every GPU-flag schedule (k_push_wait): segment sg's bytes into
// a peer's window with 16-byte write-through stores (st_wt_at: sc0 sc1, so a
// completed store is at the owner whatever cache type the writer's mapping of
// the peer window has) from a full grid, four loads in flight per lane (as
// k_copy_segs).  EVERY lane then waits until its own stores have completed
// (stores_done: s_waitcnt vmcnt(0), without the L2 writeback an agent-scope
// fence adds), the workgroup meets at a barrier, and thread 0 counts the
// workgroup done (count_done); the last one posts `seq` into every flag with a
// system-scope release -- the threadFenceReduction pattern: every
// workgroup's data completed before its count, so no flag can overtake any of
// it.  The launcher keeps every segment below 4 GiB (32-bit buffer offsets).
__device__ __forceinline__ void copy_post_body(const CopySegs& c, const PostFlags& f, unsigned* counter,
                                               unsigned total, unsigned bx, unsigned gx, int sg)
{
    const char* src = static_cast<const char*>(c.src[sg]);
    char* dst = static_cast<char*>(c.dst[sg]);
    const size_t nb = c.nbytes[sg];
    const size_t stride = (size_t)gx * 256;
    size_t done = 0;
    if ((((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        const size_t nv = nb / 16;
        const u32x4* s4 = reinterpret_cast<const u32x4*>(src);
        size_t i = (size_t)bx * 256 + threadIdx.x;
        const __amdgpu_buffer_rsrc_t r = wt_rsrc(dst);
        for (; i + 3 * stride < nv; i += 4 * stride) {
            const u32x4 a0 = s4[i], a1 = s4[i + stride], a2 = s4[i + 2 * stride], a3 = s4[i + 3 * stride];
            st_wt_at(r, 16 * i, a0); st_wt_at(r, 16 * (i + stride), a1);
            st_wt_at(r, 16 * (i + 2 * stride), a2); st_wt_at(r, 16 * (i + 3 * stride), a3);
        }
        for (; i < nv; i += stride) st_wt_at(r, 16 * i, s4[i]);
        done = nv * 16;
    }
    for (size_t i = done + (size_t)bx * 256 + threadIdx.x; i < nb; i += stride) st_wt_elem(dst + i, src[i]);
    stores_done();
    __syncthreads();
    // counter: a kCountWords block (count_done); b = this workgroup's index
    if (threadIdx.x == 0 && count_done(counter, (unsigned)sg + bx * (unsigned)c.n, total)) {
        for (int k = 0; k < f.n; ++k)
            __hip_atomic_store(f.dst[k], f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- reference-order multi-input combine ----------------------------------------
// One pass over up to 2*kMaxLeaves inputs that reproduces the association AND
// the inout/in roles of the reference's multi-step schedules:
//   tree  (chain == 0): leaf_k = pair_k ? f(s[2k], s[2k+1]) : s[2k], k < P (pow2),
//         then the balanced tree ((l0 op l1) op (l2 op l3)) op ... with the left
//         operand always in the `inout` role (recursive doubling / halving,
//         reduce.cpp:3890-4009, 1088-1175; the non-power-of-two fold is the
//         leaf pair, reduce.cpp:3835-3871);
//   chain (chain == 1): ((s0 op s1) op s2) op ... op s[P-1] (pairwise exchange,
//         reduce.cpp:1258-1318).
constexpr int kMaxLeaves = 16;
constexpr int kMaxExtraOut = 31;
struct TreeArgs {
    const void* s[2 * kMaxLeaves];
    void* extra[kMaxExtraOut];   // further destinations of the result (peer windows)
    int nextra;
    int P;
    int nleaves;   // leaves present (<= P); the rest of the P-leaf tree is empty
    unsigned pairmask;
    int chain;
    int wt;    // results announced by done_flags: write-through stores (st_wt)
    // result-ready flags (barrier-free two-step allreduce): once every tree
    // workgroup of all `done_launches` launches has stored its results, post
    // done_flags (see tree_done)
    unsigned* done_counter;       // kCountWords block: [0] count_done, [1] launches done
    unsigned done_launches;
    PostFlags done_flags;
    // tile order: 0 = XCD-contiguous eighths (the default), -1 = dispatch
    // order (the one-wave DRAM-regime geometry, msx_tree_impl.h), G > 0 = XCD
    // x owns interleaved runs of G consecutive tiles (combine_tile's orders)
    int xg;
};

// Workgroup b of nb -> tile under TreeArgs::xg (a bijection on [0, nb)).
__device__ __forceinline__ size_t tree_tile(int xg, unsigned b, unsigned nb)
{
    if (xg == 0) return xcd_tile(b, nb);
    if (xg < 0) return b;
    const unsigned g = (unsigned)xg, full = (nb / (8u * g)) * (8u * g);
    if (b >= full) return b;
    const unsigned x = b & 7, j = b >> 3;
    return ((size_t)(j / g) * 8 + x) * g + (j % g);
}

// End of a tree workgroup when the launch posts result-ready flags: the
// threadFenceReduction pattern of copy_post_body, extended over the launches
// that together evaluate one call (stream-ordered, so at most one is in
// flight).  Every lane waits for its own write-through stores (stores_done),
// thread 0 counts the workgroup, the launch's last workgroup counts the
// launch, and the last workgroup of the last launch posts the flags with
// system-scope release stores.  Both words are left zero for the next call.
__device__ __forceinline__ void tree_done(const TreeArgs& a, unsigned b, unsigned nb)
{
    stores_done();
    __syncthreads();
    if (threadIdx.x != 0) return;
    if (!count_done(a.done_counter, b, nb)) return;
    // launches of the call: word 1 of the block
    const unsigned l = __hip_atomic_fetch_add(a.done_counter + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (l != a.done_launches - 1) return;
    __hip_atomic_store(a.done_counter + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int k = 0; k < a.done_flags.n; ++k)
        __hip_atomic_store(a.done_flags.dst[k], a.done_flags.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The GPU-side wait of every flag schedule, run by ONE workgroup of a
// k_push_wait launch: thread 0 polls the peers' flags (uncached window
// memory, system-scope loads) until each reaches the call's sequence number;
// the launches after it on the stream read what the flags announce.  Only a
// single workgroup per rank ever spins, so ranks that share a GPU cannot
// starve each other's pushes.  Bounded: after
// `ticks` of s_memrealtime (100 MHz; MSX_FLAG_TIMEOUT_MS, default 20 s) it
// reports through *wait_err -- tag * 65536 + 1 + the first peer whose flag is
// missing, so the host can name the phase and the peer -- and the workgroup
// exits, so a missing peer can never leave a wave running.
__device__ __forceinline__ bool wait_flags_body(const unsigned long long* flags, unsigned long long seq, int n,
                                                int skip, int* err, unsigned long long ticks, int tag)
{
    __shared__ int ok;
    if (threadIdx.x == 0) {
        int good = 1;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        for (int r = 0; r < n && good; ++r) {
            if (r == skip) continue;
            while (__hip_atomic_load(flags + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
                    __hip_atomic_store(err, tag * 65536 + 1 + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    good = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        // The acquire that pairs with the pusher's system-scope release of the
        // flag: invalidates this CU's L1 and the XCD's L2 copies of peer-written
        // lines, so the IN half is read fresh whatever cache type the window
        // is mapped with (the UC mapping makes it a no-op for the data today,
        // but the kernel no longer depends on that allocation property).
        if (good) (void)__hip_atomic_load(flags, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

template <class F, class V, class LD>
__device__ __forceinline__ V tree_eval(const TreeArgs& a, LD load)
{
    if (a.chain) {
        // every source loaded before the first combine (the loop bound is a
        // runtime value: a rolled loop waited for each load in turn, 75 us
        // instead of 8 us for a 4-rank 1 MiB reduce_scatter); same order
        V x[kMaxLeaves];
#pragma unroll
        for (int k = 0; k < kMaxLeaves; ++k)
            if (k < a.P) x[k] = load(k);
        V v = x[0];
#pragma unroll
        for (int k = 1; k < kMaxLeaves; ++k)
            if (k < a.P) v = F::apply(v, x[k]);
        return v;
    }
    // leaves >= nleaves are absent (binomial trees over a non-power-of-two p):
    // a node whose right subtree is empty passes its left value up unchanged.
    V v[kMaxLeaves];
#pragma unroll
    for (int k = 0; k < kMaxLeaves; ++k) {
        if (k < a.nleaves) {
            v[k] = load(2 * k);
            if ((a.pairmask >> k) & 1u) v[k] = F::apply(v[k], load(2 * k + 1));
        }
    }
#pragma unroll
    for (int w = 1; w < kMaxLeaves; w *= 2) {
#pragma unroll
        for (int k = 0; k + w < kMaxLeaves; k += 2 * w)
            if (k + w < a.nleaves) v[k] = F::apply(v[k], v[k + w]);
    }
    return v[0];
}

// Result vector i into `out` and every extra destination; write-through when
// done_flags will announce it to other GPUs (TreeArgs::wt).
__device__ __forceinline__ void put_vec(const TreeArgs& a, u32x4* __restrict__ out, size_t i, u32x4 r)
{
    if (a.wt) {
        st_wt_at(wt_rsrc(out), 16 * i, r);
        for (int e = 0; e < a.nextra; ++e) st_wt_at(wt_rsrc(a.extra[e]), 16 * i, r);
    } else {
        out[i] = r;
        for (int e = 0; e < a.nextra; ++e) reinterpret_cast<u32x4*>(a.extra[e])[i] = r;
    }
}

template <int OP, class VT> struct VecFn {
    __device__ static u32x4 apply(u32x4 io, u32x4 in) { return apply_vec<OP, VT>(io, in); }
};

// The full balanced tree over NL sources (no pairs, no absent leaves: every
// power-of-two p of the allreduce / reduce_scatter / reduce trees), or with
// CHAIN the left-deep chain over NL sources (pairwise exchange), with the
// source count known at compile time: no runtime leaf tests, NL*U source
// vectors per lane issued before the first combine, tiles of BLOCK*U vectors.
// Same association and operand roles as tree_vec / tree_eval.  The generic
// kernel's runtime leaf tests cost 25 % (p = 8, fp32 SUM, 32 MiB per source:
// 55 us generic vs 44.6 us here, profiles/r02/tree_probe.json).
//
// MASKED (trees only): the same NL-leaf tree with the non-power-of-two fold's
// leaf pairs (pairmask: leaf k = f(s[2k], s[2k+1])) taken at run time -- NL,
// the unrolling and the up-front loads stay compile-time, the pattern is a
// wave-uniform test per leaf (scalar branches, no divergence), so p = 3, 5, 6,
// 7 run the fixed form instead of the generic kernel's 16-leaf loop.
// run_tree_sel (msx_tree_impl.h) sends it only full-leaf trees (nleaves ==
// P); trees with absent leaves (the rooted binomial trees) keep the generic
// kernel, which measured faster for them.
template <class F, int NL, int U, int BLOCK, bool NT, bool CHAIN, bool MASKED = false>
__device__ __forceinline__ void tree_fixed(const TreeArgs& a, u32x4* __restrict__ out, size_t nvec, size_t bid,
                                           size_t nb)
{
    static_assert(!(CHAIN && MASKED), "a chain has no pairs or absent leaves");
    constexpr size_t TILE = (size_t)BLOCK * U;
    const u32x4* src[NL];
    const u32x4* src2[MASKED ? NL : 1];
#pragma unroll
    for (int k = 0; k < NL; ++k)   // tree leaf k sits in slot 2k (slot 2k+1: its pair); chain source k in slot k
        src[k] = reinterpret_cast<const u32x4*>(a.s[CHAIN ? k : 2 * k]);
    if constexpr (MASKED) {
#pragma unroll
        for (int k = 0; k < NL; ++k) src2[k] = reinterpret_cast<const u32x4*>(a.s[2 * k + 1]);
    }
    const unsigned pm = MASKED ? a.pairmask : 0u;
    const int nl = MASKED ? a.nleaves : NL;
    auto reduce = [&](u32x4* v, const u32x4* w) {
        if constexpr (CHAIN) {
#pragma unroll
            for (int k = 1; k < NL; ++k) v[0] = F::apply(v[0], v[k]);
        } else {
            if constexpr (MASKED) {
#pragma unroll
                for (int k = 0; k < NL; ++k) {
                    const u32x4 f = F::apply(v[k], w[k]);
                    if ((pm >> k) & 1u) v[k] = f;
                }
            }
#pragma unroll
            for (int d = 1; d < NL; d *= 2) {
#pragma unroll
                for (int k = 0; k + d < NL; k += 2 * d) {
                    if constexpr (MASKED) {
                        const u32x4 f = F::apply(v[k], v[k + d]);
                        if (k + d < nl) v[k] = f;
                    } else {
                        v[k] = F::apply(v[k], v[k + d]);
                    }
                }
            }
        }
        return v[0];
    };
    // Every load unconditional: a load under a (uniform) branch makes hipcc
    // wait for it before the join, one dependent round trip per source
    // (measured: p = 7 binomial at 128 MiB/source 337 us with guarded loads
    // vs 180 us for the generic kernel).  Unpaired leaves load their own
    // vector again as the "pair" and absent leaves leaf 0's (the launcher
    // points those slots there): the same addresses in the same wave, served
    // by L2, not HBM; the pattern then picks results with selects.
    auto load = [&](u32x4* v, u32x4* w, size_t i) {
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            v[k] = ld<NT>(src[k] + i);
            if constexpr (MASKED) w[k] = ld<NT>(src2[k] + i);
        }
    };
    for (size_t t0 = bid * TILE; t0 < nvec; t0 += nb * TILE) {
        const size_t i0 = t0 + threadIdx.x;
        if (t0 + TILE <= nvec) {
            u32x4 v[U][NL], w[U][MASKED ? NL : 1];
#pragma unroll
            for (int u = 0; u < U; ++u) load(v[u], w[u], i0 + (size_t)u * BLOCK);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u32x4 r = reduce(v[u], w[u]);
                put_vec(a, out, i0 + (size_t)u * BLOCK, r);
            }
        } else {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const size_t i = i0 + (size_t)u * BLOCK;
                if (i < nvec) {
                    u32x4 v[NL], w[MASKED ? NL : 1];
                    load(v, w, i);
                    const u32x4 r = reduce(v, w);
                    put_vec(a, out, i, r);
                }
            }
        }
    }
}

// The generic kernel (NL == 0: any P <= 16 tree with pairs and absent
// leaves, any chain) loads the sources as the tree consumes them (tree_eval):
// p = 8 fp32 SUM, 32 MiB per source, that measured 51.7 us against 57.1 us
// with every source vector loaded up front (146 VGPRs instead of 77, half the
// waves per SIMD; round-2 tuning sweep).  NL > 0: tree_fixed.
// NT: non-temporal source loads.
template <int OP, class T, class VT, int BLOCK, bool NT = false, int NL = 0, int U = 1,
          bool CHAIN = false, bool MASKED = false>
__global__ __launch_bounds__(BLOCK) void k_tree(TreeArgs a, T* __restrict__ out, size_t nvec,
                                                size_t tail, int vec_ok)
{
    constexpr size_t EPV = 16 / sizeof(T);
    const unsigned b = blockIdx.x, nb = gridDim.x;
    const size_t stride = (size_t)nb * BLOCK;
    const size_t bid = tree_tile(a.xg, b, nb);   // XCD-contiguous by default (see combine_body)
    if constexpr (NL > 0) {
        if (vec_ok)
            tree_fixed<VecFn<OP, VT>, NL, U, BLOCK, NT, CHAIN, MASKED>(a, reinterpret_cast<u32x4*>(out), nvec, bid, nb);
    } else if (vec_ok) {
        for (size_t i = bid * BLOCK + threadIdx.x; i < nvec; i += stride) {
            auto load = [&](int k) { return ld<NT>(reinterpret_cast<const u32x4*>(a.s[k]) + i); };
            const u32x4 r = tree_eval<VecFn<OP, VT>, u32x4>(a, load);
            put_vec(a, reinterpret_cast<u32x4*>(out), i, r);
        }
    }
    const size_t first = vec_ok ? nvec * EPV : 0;
    const size_t nsc = vec_ok ? tail : tail + nvec * EPV;
    for (size_t s = (size_t)b * BLOCK + threadIdx.x; s < nsc; s += stride) {
        auto load = [&](int k) { return reinterpret_cast<const T*>(a.s[k])[first + s]; };
        const T r = tree_eval<Fn<OP>, T>(a, load);
        if (a.wt) {
            st_wt_elem(out + first + s, r);
            for (int e = 0; e < a.nextra; ++e) st_wt_elem(static_cast<T*>(a.extra[e]) + first + s, r);
        } else {
            out[first + s] = r;
            for (int e = 0; e < a.nextra; ++e) static_cast<T*>(a.extra[e])[first + s] = r;
        }
    }
    if (a.done_counter) tree_done(a, b, nb);
}

}  // namespace dev

// host side: the per-op tree launchers (msx_tree_*.hip)
// Source bytes of one tree launch above which its loads are non-temporal:
// the 256 MiB Infinity Cache (MALL) of one MI355X.  p = 8 fp32 SUM, per-source
// MiB -> us plain / non-temporal (round 3,
// profiles/r03/tree/size_sweep/): 32: 46.7 / 47.8, 48: 85.6 / 72.5,
// 64: 117.4 / 96.6, 128: 224.3 / 189.3.
constexpr size_t kTreeNtMin = (size_t)256 << 20;
template <int OP>
hipError_t tree_dispatch(Kind k, const dev::TreeArgs& a, int ns, void* out, size_t n, hipStream_t s);

}  // namespace msx
