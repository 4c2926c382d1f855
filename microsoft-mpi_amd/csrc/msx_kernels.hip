// msx_kernels.hip — gfx950 (CDNA4) element-wise MPI_Op combine kernels.
//
// What the reference does (src/mpi/msmpi/mpid/op.cpp:14-160): a scalar loop
// `inout[i] = inout[i] (op) in[i]` per (op, C type).  What this file does:
// the same element semantics as a memory-bound stream on MI355X:
//   * 16-byte (dwordx4) coalesced loads/stores per lane; a 64-lane wave moves
//     1 KiB per instruction per operand;
//   * UNROLL independent vectors per lane per operand in flight before the
//     first use, so each CU keeps enough HBM requests outstanding
//     (MI355X_MICROARCH.md: ~10 B/cyc/CU HBM-bound dwordx4);
//   * one tile of BLOCK*UNROLL vectors per workgroup: >> 256 CUs x 8 XCDs for
//     the benchmark sizes; full tiles run with no bounds checks;
//   * head/tail elements (unaligned start, ragged end) are handled by the same
//     launch with scalar element loads, so every (pointer, count) is legal;
//   * no MFMA: arithmetic intensity is 1 op per 3 x sizeof(T) bytes.
// Numerics: compiled with -ffp-contract=off and IEEE denormals so every
// float result is the single correctly-rounded IEEE op the reference performs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <type_traits>

#include "msx_combine_dev.h"
#include "msx_kernels.h"

namespace msx {
namespace dev {

template <int OP, class T, class VT, int UNROLL, int BLOCK, bool NTLD, bool NTST>
__global__ __launch_bounds__(BLOCK) void k_combine(const T* __restrict__ in, T* __restrict__ io,
                                                   size_t head, size_t nvec, size_t tail)
{
    combine_body<OP, T, VT, UNROLL, BLOCK, NTLD, NTST>(in, io, head, nvec, tail);
}

// Same body for operands beyond the L2 (DRAM-bound): one-wave workgroups,
// and XCD x owns interleaved runs of kDramRun consecutive 1-KiB tiles (128 KiB
// of each operand), so the eight XCDs stream eight neighbouring 128-KiB
// windows: per-XCD L2 locality and few concurrent DRAM streams at once.
// Rounds 4-5 ran the same workgroups in plain dispatch order (round-robin over
// XCDs).  fp32 SUM, interleaved, 5 rounds, us back to back / cache flushed
// (scripts/combine_geometry_probe.py, profiles/r06/geometry/), dispatch
// order -> runs of 128: 128 MiB 61.1 -> 58.3 / 70.4 -> 66.4, 256 MiB 118.3 ->
// 113.4 / 137.2 -> 130.3, 512 MiB 280.9 -> 264.5 / 274.2 -> 262.2, 2 GiB
// 1096 -> 1061 / 1093 -> 1059; 1 GiB within 0.5 %.  Runs of 64, 256 and 512
// tiles, 128-lane workgroups and XCD-contiguous eighths do not beat it.
constexpr int kDramRun = 128;
template <int OP, class T, class VT, int BLOCK, bool NTLD, bool NTST>
__global__ __launch_bounds__(BLOCK) void k_combine_dram(const T* __restrict__ in, T* __restrict__ io,
                                                        size_t head, size_t nvec, size_t tail)
{
    combine_body<OP, T, VT, 1, BLOCK, NTLD, NTST, kDramRun>(in, io, head, nvec, tail);
}

// Same body, launched by the host-memory path of MPI_Reduce_local (pinned
// operands read over PCIe, or HBM staging chunks): a separate symbol so the
// rocprof statistics of the device-resident kernel stay clean.
template <int OP, class T, class VT, int UNROLL, int BLOCK, bool NTLD, bool NTST>
__global__ __launch_bounds__(BLOCK) void k_combine_host(const T* __restrict__ in, T* __restrict__ io,
                                                        size_t head, size_t nvec, size_t tail)
{
    combine_body<OP, T, VT, UNROLL, BLOCK, NTLD, NTST>(in, io, head, nvec, tail);
}

// Mutually misaligned operands, both element-aligned (e.g. sub-arrays at
// different offsets): the vector grid follows `io` (16-byte aligned), and the
// matching 16 bytes of `in`, which straddle two aligned 16-byte chunks, are
// loaded as those two chunks and realigned in registers (v_alignbyte), so
// every load stays aligned and coalesced.  `s` = byte offset of in's vector
// data from 16-byte alignment (1..15, a multiple of sizeof(T)).  Vector 0 and
// the last vector are left to the scalar loop: their outer chunk reaches
// before / past the operand.  Before this path such calls ran element by
// element: 256 MiB fp32 at 4.9 TB/s, int8 at 1.7 TB/s.
__device__ __forceinline__ u32x4 realign(const u32x4& A, const u32x4& B, unsigned s)
{
    const unsigned d[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    const unsigned r = s & 3;
    u32x4 o;
    switch (s >> 2) {
    case 0:
        o = u32x4{__builtin_amdgcn_alignbyte(d[1], d[0], r), __builtin_amdgcn_alignbyte(d[2], d[1], r),
                  __builtin_amdgcn_alignbyte(d[3], d[2], r), __builtin_amdgcn_alignbyte(d[4], d[3], r)};
        break;
    case 1:
        o = u32x4{__builtin_amdgcn_alignbyte(d[2], d[1], r), __builtin_amdgcn_alignbyte(d[3], d[2], r),
                  __builtin_amdgcn_alignbyte(d[4], d[3], r), __builtin_amdgcn_alignbyte(d[5], d[4], r)};
        break;
    case 2:
        o = u32x4{__builtin_amdgcn_alignbyte(d[3], d[2], r), __builtin_amdgcn_alignbyte(d[4], d[3], r),
                  __builtin_amdgcn_alignbyte(d[5], d[4], r), __builtin_amdgcn_alignbyte(d[6], d[5], r)};
        break;
    default:
        o = u32x4{__builtin_amdgcn_alignbyte(d[4], d[3], r), __builtin_amdgcn_alignbyte(d[5], d[4], r),
                  __builtin_amdgcn_alignbyte(d[6], d[5], r), __builtin_amdgcn_alignbyte(d[7], d[6], r)};
        break;
    }
    return o;
}

// Lane i takes lane i+1's word: DPP wave_shl:1 (a VALU operand modifier on
// the GFX9 family, dpp_ctrl 0x130).  Lane 63 gets 0; it loads its own next
// chunk.  A ds_bpermute through the LDS crossbar measured the same (within
// 0.5 %, profiles/r03/misalign/misalign_ab_box2.json).
__device__ __forceinline__ unsigned from_next_lane(unsigned x)
{
    return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x130, 0xf, 0xf, true);
}

template <int OP, class T, class VT, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_combine_shift(const T* __restrict__ in, T* __restrict__ io, size_t head,
                                                         size_t nvec, size_t tail, unsigned s)
{
    constexpr size_t EPV = 16 / sizeof(T);
    const u32x4* __restrict__ ain =
        reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(in + head) - s);   // aligned
    u32x4* __restrict__ vio = reinterpret_cast<u32x4*>(io + head);
    const size_t bid = (size_t)xcd_tile(blockIdx.x, gridDim.x);
    // vector v of lane tid: wave spans start on 1-KiB boundaries of `io`'s
    // vector grid (vector 0 is left idle, not shifted to lane 0: a grid that
    // started at vector 1 made every wave straddle one more 128-B line per
    // operand, -12 % at 256 MiB)
    const size_t v = bid * BLOCK + threadIdx.x;
    const bool live = v >= 1 && v + 1 < nvec;
    // chunk v+1 is the next lane's chunk v: taken with a lane shuffle, loaded
    // only by the wave's last lane and the last live lane
    // The extra chunk of those lanes is loaded together with the other two
    // operands, not after the shuffle: issued behind the wait for `a` it added
    // a second memory round trip to every wave (0.79 of the aligned rate).
    const bool own_next = live && ((threadIdx.x & 63) == 63 || v + 2 >= nvec);
    u32x4 a = {0, 0, 0, 0}, y = {0, 0, 0, 0}, nx = {0, 0, 0, 0};
    if (live) {
        a = ld<true>(ain + v);
        y = ld<true>(vio + v);
    }
    if (own_next) nx = ld<true>(ain + v + 1);
    asm volatile("" : "+v"(a), "+v"(y), "+v"(nx));
    __builtin_amdgcn_sched_barrier(0);
    u32x4 b;
    b.x = from_next_lane(a.x);
    b.y = from_next_lane(a.y);
    b.z = from_next_lane(a.z);
    b.w = from_next_lane(a.w);
    if (own_next) b = nx;
    if (live) vio[v] = apply_vec<OP, VT>(y, realign(a, b, s));
    // scalar: [0, head + EPV) and [head + (nvec - 1) * EPV, head + nvec * EPV + tail)
    const size_t first = head + EPV, last0 = head + (nvec - 1) * EPV;
    const size_t nscalar = first + (EPV + tail);
    for (size_t i = (size_t)blockIdx.x * BLOCK + threadIdx.x; i < nscalar; i += (size_t)gridDim.x * BLOCK) {
        const size_t e = i < first ? i : last0 + (i - first);
        io[e] = Fn<OP>::apply(io[e], in[e]);
    }
}

}  // namespace dev
}  // namespace msx

#include "msx_tree_dev.h"

namespace msx {
namespace dev {

// ---- multi-segment copy (allgather phase: blocks pulled from peers) -------------
__global__ __launch_bounds__(64) void k_post_flags(PostFlags f)
{
    if (threadIdx.x < (unsigned)f.n)
        __hip_atomic_store(f.dst[threadIdx.x], f.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void k_copy_segs(CopySegs c)
{
    // One 1-D grid, workgroup b serving segment b % n: consecutive workgroups
    // go to different segments, so the dispatcher starts every segment (every
    // peer link, when the segments are remote) at once instead of filling the
    // GPU with the first few segments' workgroups.  One 4-KiB tile per
    // workgroup and lane (16-B non-temporal loads), as the HBM probe's copy:
    // the earlier grid-stride form (<= 512 workgroups per segment, 4 loads in
    // flight per lane) copied 256 MiB locally at 5.5 TB/s of traffic, this
    // form at the probe's ~8 TB/s (profiles/r02/copy/copy_cmp.log).  A single segment
    // (a local copy) takes the XCD-contiguous tile order of the combine.
    const unsigned n = (unsigned)c.n;
    const int sg = (int)(blockIdx.x % n);
    const size_t gx = gridDim.x / n;
    const size_t bx = n == 1 ? (size_t)xcd_tile(blockIdx.x, gridDim.x) : (size_t)(blockIdx.x / n);
    const char* src = static_cast<const char*>(c.src[sg]);
    char* dst = static_cast<char*>(c.dst[sg]);
    const size_t nb = c.nbytes[sg];
    const bool vec = (((uintptr_t)src | (uintptr_t)dst) & 15) == 0;
    const size_t stride = gx * 256;
    size_t done = 0;
    if (vec) {
        const size_t nv = nb / 16;
        const u32x4* s = reinterpret_cast<const u32x4*>(src);
        u32x4* d = reinterpret_cast<u32x4*>(dst);
        for (size_t i = bx * 256 + threadIdx.x; i < nv; i += stride) d[i] = ld<true>(s + i);
        done = nv * 16;
    }
    for (size_t i = done + bx * 256 + threadIdx.x; i < nb; i += stride) dst[i] = src[i];
}

// One local copy far above the 256 MiB Infinity Cache (DRAM-bound): the
// combine's DRAM-regime geometry (k_combine_dram) -- one-wave workgroups in
// dispatch order, so the eight XCDs stream neighbouring 1-KiB tiles and DRAM
// sees two streams instead of 16.  16-byte aligned, whole vectors only.
__global__ __launch_bounds__(64) void k_copy_dram(const u32x4* __restrict__ s, u32x4* __restrict__ d, size_t nv)
{
    const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
    if (i < nv) d[i] = ld<true>(s + i);
}

// The synchronisation point of every GPU-flag schedule: workgroups [0, total)
// push (copy_post_body, segment b % n: every peer link starts at once), the
// last workgroup alone waits for the peers' flags -- one spinning workgroup
// per rank, so ranks that share a GPU never starve each other's pushes -- and
// the stream's next launches read what the flags announce.
__global__ __launch_bounds__(256) void k_push_wait(CopySegs c, PostFlags f, unsigned* counter, unsigned total,
                                                   unsigned gx, const unsigned long long* wflags,
                                                   unsigned long long wseq, int wn, int wskip, int* werr,
                                                   unsigned long long wticks, int wtag)
{
    const unsigned b = blockIdx.x;
    if (b < total) {
        copy_post_body(c, f, counter, total, b / (unsigned)c.n, gx, (int)(b % (unsigned)c.n));
        return;
    }
    // flags without data (no push workgroups): nothing to order them after,
    // so the waiting workgroup posts them before it waits
    if (total == 0 && threadIdx.x < (unsigned)f.n)
        __hip_atomic_store(f.dst[threadIdx.x], f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    (void)wait_flags_body(wflags, wseq, wn, wskip, werr, wticks, wtag);
}

}  // namespace dev

// =====================================================================================
// host-side dispatch
// =====================================================================================
namespace {

using namespace dev;

constexpr int kBlock = 256;
constexpr int kUnroll = 1;

// Bytes per operand above which the device combine takes k_combine_dram:
// 16 MiB, where the two operands outgrow the
// chip's L2 (8 x 4 MiB).  Rounds 1-4 switched only above the 256 MiB Infinity
// Cache.  fp32 SUM, HIP events, interleaved (round-4 size sweep,
// profiles/r04/combine_geometry/), XCD-contiguous tiles -> dispatch order,
// GB/s back to back / with the Infinity Cache flushed first:
//    16 MiB 7077 -> 6560 / 4309 -> 4280 (L2-resident: tiles stay)
//    32 MiB 6357 -> 6614 / 4954 -> 5287     64 MiB 6221 -> 6458 / 5216 -> 5599
//   128 MiB 6639 -> 6742 / 5298 -> 6031    192 MiB 6926 -> 6864 / 5609 -> 6106
//   256 MiB 7114 -> 6999 / 5751 -> 6097
// Dispatch order wins cold at every size above L2 (+5-14 %) and back to back
// up to 128 MiB; from 160 MiB, back to back on the same operands, the
// Infinity Cache replays part of each launch and the tiles are 0.4-1.6 %
// ahead.  Operands that size are rarely still cached when a reduction comes.
size_t combine_dram_min()
{
    static const size_t v = [] {
        size_t b = (size_t)16 << 20;
        // test hook: 0 runs the DRAM-regime kernel at every size (its parity test)
        if (const char* e = getenv("MSX_TEST_COMBINE_DRAM_MIN")) b = (size_t)atoll(e);
        return b;
    }();
    return v;
}

// The realigning path (k_combine_shift): both operands element-aligned but
// at different offsets from 16-byte alignment, and at least 3 vectors.
template <class T>
inline bool split_shift(const void* in, const void* io, size_t count, size_t& head, size_t& nvec, size_t& tail,
                        unsigned& s)
{
    constexpr size_t ES = sizeof(T);
    const uintptr_t a = (uintptr_t)in, b = (uintptr_t)io;
    if (ES >= 16 || (16 % ES) != 0 || (a & 15) == (b & 15) || (a % ES) != 0 || (b % ES) != 0) return false;
    const size_t h = ((16 - (b & 15)) & 15) / ES;
    if (h >= count) return false;
    const size_t epv = 16 / ES;
    const size_t nv = (count - h) / epv;
    if (nv < 3) return false;
    head = h;
    nvec = nv;
    tail = count - h - nv * epv;
    s = (unsigned)((a + h * ES) & 15);
    return true;
}

template <int OP, class T, class VT, int UNROLL, int BLOCK, bool NTLD, bool NTST>
hipError_t run_combine(const void* in, void* io, size_t count, hipStream_t s, const LaunchCfg& cfg)
{
    size_t head, nvec, tail;
    unsigned sh = 0;
    if (split_shift<T>(in, io, count, head, nvec, tail, sh)) {
        size_t grid = (nvec + BLOCK - 1) / BLOCK;
        const size_t sc = (head + tail + 2 * (16 / sizeof(T)) + BLOCK - 1) / BLOCK;
        if (grid < sc) grid = sc;
        if (grid > 0x7fffffffu) return hipErrorInvalidValue;
        hipLaunchKernelGGL((k_combine_shift<OP, T, VT, BLOCK>), dim3((unsigned)grid), dim3(BLOCK), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(io), head, nvec, tail, sh);
        return hipGetLastError();
    }
    combine_split<T>(in, io, count, head, nvec, tail);
    if (!cfg.host && UNROLL == 1 && nvec * 16 > combine_dram_min()) {
        constexpr int DB = 64;
        size_t grid = (nvec + DB - 1) / DB;
        const size_t sc = (head + tail + DB - 1) / DB;
        if (grid < sc) grid = sc;
        if (grid > 0x7fffffffu) return hipErrorInvalidValue;    // > 2^37 bytes per operand
        hipLaunchKernelGGL((k_combine_dram<OP, T, VT, DB, NTLD, NTST>), dim3((unsigned)grid), dim3(DB), 0, s,
                           static_cast<const T*>(in), static_cast<T*>(io), head, nvec, tail);
        return hipGetLastError();
    }
    const size_t tile = (size_t)BLOCK * UNROLL;
    size_t grid = (nvec + tile - 1) / tile;
    const size_t sc = (head + tail + BLOCK - 1) / BLOCK;
    if (grid < sc) grid = sc;
    if (grid == 0) return hipSuccess;
    if (grid > 0x7fffffffu) grid = 0x7fffffffu;
    if (cfg.host)
        hipLaunchKernelGGL((k_combine_host<OP, T, VT, UNROLL, BLOCK, NTLD, NTST>), dim3((unsigned)grid),
                           dim3(BLOCK), 0, s, static_cast<const T*>(in), static_cast<T*>(io), head,
                           nvec, tail);
    else
        hipLaunchKernelGGL((k_combine<OP, T, VT, UNROLL, BLOCK, NTLD, NTST>), dim3((unsigned)grid),
                           dim3(BLOCK), 0, s, static_cast<const T*>(in), static_cast<T*>(io), head,
                           nvec, tail);
    return hipGetLastError();
}

// Default launch of every (op, type): one 16-B vector per lane per operand,
// 256-thread workgroups (one-shot grid, 65536 workgroups at 256 MiB fp32),
// non-temporal loads.  Measured on MI355X for the 256 MiB fp32 SUM
// (profiles/r01/bench_sweep.log): 7.05 TB/s vs 6.8 TB/s at 4 vectors per lane
// and 5.5 TB/s with default-policy loads.
template <int OP, class T>
hipError_t run_default(const void* in, void* io, size_t count, hipStream_t s, const LaunchCfg& cfg)
{
    return run_combine<OP, T, T, kUnroll, kBlock, true, false>(in, io, count, s, cfg);
}

// Bitwise ops: byte-granular scalars, 32-bit lanes inside vectors.
template <int OP>
hipError_t run_bitwise(const void* in, void* io, size_t nbytes, hipStream_t s, const LaunchCfg& cfg)
{
    return run_combine<OP, uint8_t, uint32_t, kUnroll, kBlock, true, false>(in, io, nbytes, s, cfg);
}

template <int OP>
hipError_t dispatch_arith(Kind k, const void* in, void* io, size_t n, hipStream_t s,
                          const LaunchCfg& c)
{
    switch (k) {
    case K_I8:  return run_default<OP, int8_t>(in, io, n, s, c);
    case K_U8:  return run_default<OP, uint8_t>(in, io, n, s, c);
    case K_I16: return run_default<OP, int16_t>(in, io, n, s, c);
    case K_U16: return run_default<OP, uint16_t>(in, io, n, s, c);
    case K_I32: return run_default<OP, int32_t>(in, io, n, s, c);
    case K_U32: return run_default<OP, uint32_t>(in, io, n, s, c);
    case K_I64: return run_default<OP, int64_t>(in, io, n, s, c);
    case K_U64: return run_default<OP, uint64_t>(in, io, n, s, c);
    case K_F32: return run_default<OP, float>(in, io, n, s, c);
    case K_F64: return run_default<OP, double>(in, io, n, s, c);
    default: break;
    }
    if constexpr (OP == O_SUM || OP == O_PROD) {
        if (k == K_C32) return run_default<OP, c32>(in, io, n, s, c);
        if (k == K_C64) return run_default<OP, c64>(in, io, n, s, c);
    }
    if constexpr (OP == O_LAND || OP == O_LOR || OP == O_LXOR) {
        if (k == K_BOOL) return run_default<OP, uint8_t>(in, io, n, s, c);
    }
    return hipErrorInvalidValue;
}

template <int OP>
hipError_t dispatch_loc(Kind k, const void* in, void* io, size_t n, hipStream_t s,
                        const LaunchCfg& c)
{
    switch (k) {
    case K_LOC_II: return run_default<OP, loc_ii>(in, io, n, s, c);
    case K_LOC_FI: return run_default<OP, loc_fi>(in, io, n, s, c);
    case K_LOC_SI: return run_default<OP, loc_si>(in, io, n, s, c);
    case K_LOC_DI: return run_default<OP, loc_di>(in, io, n, s, c);
    case K_LOC_FF: return run_default<OP, loc_ff>(in, io, n, s, c);
    case K_LOC_DD: return run_default<OP, loc_dd>(in, io, n, s, c);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_combine(int opidx, Kind k, const void* in, void* io, size_t n, hipStream_t s,
                          const LaunchCfg& c)
{
    if (n == 0) return hipSuccess;
    switch (opidx) {
    case O_SUM:  return dispatch_arith<O_SUM>(k, in, io, n, s, c);
    case O_MAX:  return dispatch_arith<O_MAX>(k, in, io, n, s, c);
    case O_MIN:  return dispatch_arith<O_MIN>(k, in, io, n, s, c);
    case O_PROD: return dispatch_arith<O_PROD>(k, in, io, n, s, c);
    case O_LAND: return dispatch_arith<O_LAND>(k, in, io, n, s, c);
    case O_LOR:  return dispatch_arith<O_LOR>(k, in, io, n, s, c);
    case O_LXOR: return dispatch_arith<O_LXOR>(k, in, io, n, s, c);
    case O_BAND: return run_bitwise<O_BAND>(in, io, n * kind_size(k), s, c);
    case O_BOR:  return run_bitwise<O_BOR>(in, io, n * kind_size(k), s, c);
    case O_BXOR: return run_bitwise<O_BXOR>(in, io, n * kind_size(k), s, c);
    case O_MAXLOC: return dispatch_loc<O_MAXLOC>(k, in, io, n, s, c);
    case O_MINLOC: return dispatch_loc<O_MINLOC>(k, in, io, n, s, c);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_tree(int opidx, Kind k, const void* const* srcs, int p, void* out, size_t n,
                       hipStream_t s)
{
    // Plain balanced tree over p (power of two) inputs, no pairs.
    if (p < 1 || p > kMaxLeaves || (p & (p - 1))) return hipErrorInvalidValue;
    TreeSpec t;
    t.P = p;
    t.pairmask = 0;
    t.chain = false;
    for (int i = 0; i < p; ++i) t.src[2 * i] = srcs[i];
    return launch_tree_spec(opidx, k, t, out, n, s);
}

hipError_t launch_tree_spec(int opidx, Kind k, const TreeSpec& t, void* out, size_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    if (t.P < 1 || t.P > kMaxLeaves) return hipErrorInvalidValue;
    TreeArgs a{};
    int ns;
    if (t.chain) {
        for (int i = 0; i < t.P; ++i) a.s[i] = t.src[i];
        ns = t.P;
    } else {
        if (t.P & (t.P - 1)) return hipErrorInvalidValue;
        for (int i = 0; i < 2 * t.P; ++i) a.s[i] = t.src[i];
        ns = 0;
        const int nl = (t.nleaves > 0 && t.nleaves <= t.P) ? t.nleaves : t.P;
        // absent leaves read leaf 0's source (tree_fixed MASKED loads every slot; the
        // same addresses in the same wave hit L2) and never use it
        for (int i = nl; i < t.P; ++i) a.s[2 * i] = a.s[2 * i + 1] = t.src[0];
        for (int i = 0; i < nl; ++i) {
            if (!t.src[2 * i]) return hipErrorInvalidValue;
            if ((t.pairmask >> i) & 1u) { if (!t.src[2 * i + 1]) return hipErrorInvalidValue; }
            else a.s[2 * i + 1] = t.src[2 * i];   // unpaired: the leaf's own source (read, not used)
        }
        ns = 2 * t.P;
    }
    if (t.nextra < 0 || t.nextra > kMaxExtraOut) return hipErrorInvalidValue;
    a.nextra = t.nextra;
    for (int e = 0; e < t.nextra; ++e) a.extra[e] = t.extra[e];
    a.P = t.P;
    a.nleaves = (t.nleaves > 0 && t.nleaves <= t.P) ? t.nleaves : t.P;
    a.pairmask = t.pairmask;
    a.chain = t.chain ? 1 : 0;
    if (t.done_counter) {
        if (t.done_nflags < 0 || t.done_nflags > 64 || t.done_launches < 1) return hipErrorInvalidValue;
        a.done_counter = t.done_counter;
        // results that result-ready flags announce to peers: write-through
        // stores (buffer-store offsets are 32-bit: larger ranges keep plain
        // stores; the two-step chunks stay far below 4 GiB)
        a.wt = n * kind_size(k) < ((size_t)1 << 32) ? 1 : 0;
        a.done_launches = t.done_launches;
        a.done_flags.n = t.done_nflags;
        a.done_flags.seq = t.done_seq;
        for (int i = 0; i < t.done_nflags; ++i) a.done_flags.dst[i] = t.done_flags[i];
    }
    if (!t.chain && t.P == 1 && t.pairmask == 0 && t.nextra == 0 && !t.done_counter) {
        if (t.src[0] == out) return hipSuccess;
        return hipMemcpyAsync(out, t.src[0], n * kind_size(k), hipMemcpyDeviceToDevice, s);   // xfer: device/pinned
    }
    switch (opidx) {
    case O_SUM:    return tree_dispatch<O_SUM>(k, a, ns, out, n, s);
    case O_MAX:    return tree_dispatch<O_MAX>(k, a, ns, out, n, s);
    case O_MIN:    return tree_dispatch<O_MIN>(k, a, ns, out, n, s);
    case O_PROD:   return tree_dispatch<O_PROD>(k, a, ns, out, n, s);
    case O_LAND:   return tree_dispatch<O_LAND>(k, a, ns, out, n, s);
    case O_LOR:    return tree_dispatch<O_LOR>(k, a, ns, out, n, s);
    case O_LXOR:   return tree_dispatch<O_LXOR>(k, a, ns, out, n, s);
    case O_BAND:   return tree_dispatch<O_BAND>(k, a, ns, out, n, s);
    case O_BOR:    return tree_dispatch<O_BOR>(k, a, ns, out, n, s);
    case O_BXOR:   return tree_dispatch<O_BXOR>(k, a, ns, out, n, s);
    case O_MAXLOC: return tree_dispatch<O_MAXLOC>(k, a, ns, out, n, s);
    case O_MINLOC: return tree_dispatch<O_MINLOC>(k, a, ns, out, n, s);
    default: return hipErrorInvalidValue;
    }
}

unsigned long long flag_wait_ticks()
{
    static const unsigned long long t = [] {
        const char* e = getenv("MSX_FLAG_TIMEOUT_MS");
        long long ms = e ? atoll(e) : 20000;
        if (ms < 1) ms = 1;
        return (unsigned long long)ms * 100000ull;          // s_memrealtime: 100 MHz
    }();
    return t;
}

double flag_wait_seconds() { return (double)flag_wait_ticks() / 1e8; }

hipError_t launch_push_wait(const void* const* src, void* const* dst, const size_t* nbytes, int nseg,
                            unsigned long long* const* flags, int nflags, unsigned long long seq,
                            unsigned* counter, const unsigned long long* wait_flags, int wait_n, int wait_skip,
                            int* wait_err, hipStream_t s, int wait_tag)
{
    if (nseg < 0 || nseg > kMaxSegs || nflags < 0 || nflags > 64 || !wait_flags || !wait_err ||
        (nseg > 0 && !counter))
        return hipErrorInvalidValue;
    CopySegs c{};
    PostFlags f{};
    size_t maxb = 0;
    c.n = nseg > 0 ? nseg : 1;
    for (int i = 0; i < nseg; ++i) {
        c.src[i] = src[i];
        c.dst[i] = dst[i];
        c.nbytes[i] = nbytes[i];
        if (nbytes[i] > maxb) maxb = nbytes[i];
    }
    if (maxb >= ((size_t)1 << 32)) return hipErrorInvalidValue;   // 32-bit write-through offsets
    f.n = nflags;
    f.seq = seq;
    for (int i = 0; i < nflags; ++i) f.dst[i] = flags[i];
    // One 16-byte granule per lane and pass, at most kPushGridCap pushing
    // workgroups in all: the copy kernel's geometry.  Rounds 1-3 used four
    // granules per lane and 2048 workgroups, which measured the same up to
    // 64 MiB (profiles/r02/copy/push_cmp.log) but 4-7 % slower at c3/c4 sizes
    // once the chunks were pipelined (round-4 A/B,
    // profiles/r04/pushab/).
    constexpr size_t kPushGridCap = 65536;
    size_t gx = (maxb / 16 + 255) / 256;
    const size_t cap = nseg > 0 ? std::max<size_t>(1, kPushGridCap / (size_t)nseg) : 1;
    if (gx < 1) gx = 1;
    if (gx > cap) gx = cap;
    const unsigned total = nseg > 0 ? (unsigned)(gx * (size_t)nseg) : 0u;
    hipLaunchKernelGGL(k_push_wait, dim3(total + 1), dim3(256), 0, s, c, f, counter, total,
                       (unsigned)gx, wait_flags, seq, wait_n, wait_skip, wait_err, flag_wait_ticks(), wait_tag);
    return hipGetLastError();
}

hipError_t launch_post_flags(unsigned long long* const* dst, int n, unsigned long long seq, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    if (n > 64) return hipErrorInvalidValue;
    PostFlags f{};
    for (int i = 0; i < n; ++i) f.dst[i] = dst[i];
    f.seq = seq;
    f.n = n;
    hipLaunchKernelGGL(k_post_flags, dim3(1), dim3(64), 0, s, f);
    return hipGetLastError();
}

// Bytes of one local copy above which it takes k_copy_dram: 16 MiB, as the
// combine (combine_dram_min).  Rounds 1-4 switched above
// 256 MiB.  HIP events, interleaved (round-4 probe,
// profiles/r04/combine_geometry/copy.json), tiles -> dispatch order, GB/s back
// to back / cache flushed: 16 MiB 4637 -> 4284 / 3277 -> 3452 (tiles stay),
// 32 MiB 4981 -> 5384 / 4153 -> 4427, 64 MiB 5696 -> 6025 / 4706 -> 5335,
// 128 MiB 6475 -> 6822 / 5247 -> 5780, 256 MiB 7150 -> 7259 / 5836 -> 6237.
constexpr size_t kCopyDramMin = (size_t)16 << 20;

hipError_t launch_copy_segs(const void* const* src, void* const* dst, const size_t* nbytes, int nseg,
                            hipStream_t s)
{
    // one local copy in the DRAM regime (the collect of a 512 MiB chunk)
    if (nseg == 1 && nbytes[0] > kCopyDramMin && ((((uintptr_t)src[0] | (uintptr_t)dst[0] | nbytes[0]) & 15) == 0)) {
        const size_t nv = nbytes[0] / 16, grid = (nv + 63) / 64;
        if (grid > 0x7fffffffu) return hipErrorInvalidValue;
        hipLaunchKernelGGL(k_copy_dram, dim3((unsigned)grid), dim3(64), 0, s, static_cast<const u32x4*>(src[0]),
                           static_cast<u32x4*>(dst[0]), nv);
        return hipGetLastError();
    }
    for (int base = 0; base < nseg; base += kMaxSegs) {
        CopySegs c{};
        c.n = (nseg - base < kMaxSegs) ? nseg - base : kMaxSegs;
        size_t maxb = 0;
        for (int i = 0; i < c.n; ++i) {
            c.src[i] = src[base + i];
            c.dst[i] = dst[base + i];
            c.nbytes[i] = nbytes[base + i];
            if (c.nbytes[i] > maxb) maxb = c.nbytes[i];
        }
        if (maxb == 0) continue;
        // one 4-KiB tile per workgroup, grid-stride beyond 2^22 workgroups in all
        constexpr size_t cap = (size_t)1 << 22;
        size_t gx = (maxb / 16 + 255) / 256;
        if (gx < 1) gx = 1;
        size_t gmax = cap / (size_t)c.n;
        if (gmax < 1) gmax = 1;
        if (gx > gmax) gx = gmax;
        hipLaunchKernelGGL(k_copy_segs, dim3((unsigned)(gx * (size_t)c.n)), dim3(256), 0, s, c);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace msx
