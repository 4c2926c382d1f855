// msx_pack.hip — gfx950 kernels of the derived-datatype engine (msx_dtype.h).
//
// The reference interprets a dataloop tree on the CPU, one contiguous piece at
// a time (MPID_Segment_pack / unpack, mpid/segment.cpp; the accumulate walk of
// packethandling.cpp:2969-3004).  Here a committed type is a flat list of byte
// runs, and every work item maps one packed granule straight to its typed
// address:
//
//   packed byte p of instance i  ->  typed[i*extent + disp[k] + (p - poff[k])]
//
// with k found by a magic-number division for regular layouts (vector,
// hvector, subarray rows: run k = first + k*stride) and by a binary search
// over the run offsets otherwise.  The granule G is the largest power of two
// <= 16 that divides every run offset / length, the size, the extent and both
// pointers, so a granule never straddles two runs and every access is a
// naturally aligned G-byte load or store.  The kernels are HBM-bound byte
// movers (no arithmetic beyond the address map); a pack moves 2*size bytes per
// instance.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "msx_dev_ops.h"
#include "msx_dtype.h"
#include "msx_kernels.h"

namespace msx {
namespace dev {

// q = n / d for any 32-bit n (Granlund-Montgomery round-up method).
struct FastDiv {
    uint32_t d = 1, m = 0, s = 0;
    FastDiv() = default;
    explicit FastDiv(uint32_t div) : d(div)
    {
        s = 0;
        while ((1ull << s) < div) ++s;
        m = (uint32_t)((((1ull << 32) * ((1ull << s) - div)) / div) + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const
    {
        return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> s);
    }
};

struct CopyArgs {
    char* typed;
    char* packed;
    int64_t ngran;           // granules in the packed stream (count * size / G)
    int64_t extent;          // bytes
    int64_t size;            // bytes per instance
    // regular layout, in granules where noted
    int64_t first;           // bytes
    int64_t stride;          // bytes
    int64_t gsize, gblen;    // granules
    FastDiv fd_size, fd_blen;
    // two-level regular layout (n1 > 0): run k at first + (k / n1)*stride2 + (k % n1)*stride
    int64_t n1, stride2;
    FastDiv fd_n1;
    // general layout
    const int64_t* disp;
    const int64_t* poff;
    int64_t nruns;
};

constexpr int kPackBlock = 256;

template <int G> struct GranT;
template <> struct GranT<1> { typedef uint8_t T; };
template <> struct GranT<2> { typedef uint16_t T; };
template <> struct GranT<4> { typedef uint32_t T; };
template <> struct GranT<8> { typedef uint64_t T; };
template <> struct GranT<16> { typedef u32x4 T; };

// Largest k with poff[k] <= q (poff[0] = 0, poff[nruns] = size > q).
__device__ __forceinline__ int64_t find_run(const int64_t* __restrict__ poff, int64_t nruns, int64_t q)
{
    int64_t lo = 0, hi = nruns;      // invariant: poff[lo] <= q < poff[hi]
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) >> 1;
        if (poff[mid] <= q) lo = mid; else hi = mid;
    }
    return lo;
}

// Byte offset (from the typed base) of packed granule g.
template <int G, bool REG, bool NARROW>
__device__ __forceinline__ int64_t typed_off(const CopyArgs& a, int64_t g)
{
    int64_t i, q;
    if constexpr (NARROW) {
        const uint32_t gi = (uint32_t)a.fd_size.div((uint32_t)g);
        i = gi;
        q = g - (int64_t)gi * a.gsize;
    } else {
        i = g / a.gsize;
        q = g - i * a.gsize;
    }
    if constexpr (REG) {
        int64_t k;
        if constexpr (NARROW) k = a.fd_blen.div((uint32_t)q);
        else k = q / a.gblen;
        const int64_t off = q - k * a.gblen;
        if (a.n1) {             // two levels (uniform branch: a kernel argument)
            int64_t k1;
            if constexpr (NARROW) k1 = a.fd_n1.div((uint32_t)k);
            else k1 = k / a.n1;
            return i * a.extent + a.first + k1 * a.stride2 + (k - k1 * a.n1) * a.stride + off * G;
        }
        return i * a.extent + a.first + k * a.stride + off * G;
    } else {
        const int64_t qb = q * G;
        const int64_t k = find_run(a.poff, a.nruns, qb);
        return i * a.extent + a.disp[k] + (qb - a.poff[k]);
    }
}

// Granules per lane in flight: every lane issues kUnroll independent loads
// before its first store (a lone load -> store chain per lane leaves too few
// bytes in flight per CU to cover HBM latency).
constexpr int kUnroll = 4;

template <int G, bool REG, bool NARROW, bool UNPACK>
__global__ __launch_bounds__(kPackBlock) void k_dt_pack(CopyArgs a)
{
    typedef typename GranT<G>::T T;
    const int64_t stride = (int64_t)gridDim.x * kPackBlock;
    const int64_t bid = xcd_tile(blockIdx.x, gridDim.x);
    for (int64_t g0 = bid * kPackBlock + threadIdx.x; g0 < a.ngran; g0 += stride * kUnroll) {
        T v[kUnroll];
        int64_t off[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t g = g0 + u * stride;
            if (g < a.ngran) {
                off[u] = typed_off<G, REG, NARROW>(a, g);
                if constexpr (UNPACK) v[u] = __builtin_nontemporal_load(reinterpret_cast<const T*>(a.packed) + g);
                else v[u] = *reinterpret_cast<const T*>(a.typed + off[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t g = g0 + u * stride;
            if (g < a.ngran) {
                if constexpr (UNPACK) *reinterpret_cast<T*>(a.typed + off[u]) = v[u];
                else __builtin_nontemporal_store(v[u], reinterpret_cast<T*>(a.packed) + g);
            }
        }
    }
}

// Tile form for spans far above the 256 MiB Infinity Cache (the combine's
// DRAM-regime geometry, k_combine_dram): one-wave workgroups in dispatch
// order, each owning kUnroll x 64 consecutive granules, so the eight XCDs
// stream neighbouring tiles of both sides instead of the grid-stride form's
// 4 x 8 streams per side.  Same map, loads before stores, same cache policy.
template <int G, bool REG, bool NARROW, bool UNPACK>
__global__ __launch_bounds__(64) void k_dt_pack_tile(CopyArgs a)
{
    typedef typename GranT<G>::T T;
    const int64_t g0 = (int64_t)blockIdx.x * (64 * kUnroll) + threadIdx.x;
    T v[kUnroll];
    int64_t off[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const int64_t g = g0 + u * 64;
        if (g < a.ngran) {
            off[u] = typed_off<G, REG, NARROW>(a, g);
            if constexpr (UNPACK) v[u] = __builtin_nontemporal_load(reinterpret_cast<const T*>(a.packed) + g);
            else v[u] = *reinterpret_cast<const T*>(a.typed + off[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const int64_t g = g0 + u * 64;
        if (g < a.ngran) {
            if constexpr (UNPACK) *reinterpret_cast<T*>(a.typed + off[u]) = v[u];
            else __builtin_nontemporal_store(v[u], reinterpret_cast<T*>(a.packed) + g);
        }
    }
}

// Run-parallel form for layouts whose runs are long (subarray rows, big
// indexed blocks): one wavefront per (instance, run) unit, its 64 lanes
// stream the run's granules with coalesced accesses on both sides.  No
// per-granule search: the run's offsets are read once per wave.
template <int G, bool UNPACK>
__global__ __launch_bounds__(kPackBlock) void k_dt_runs(CopyArgs a)
{
    typedef typename GranT<G>::T T;
    constexpr int kWaves = kPackBlock / 64;
    const int lane = threadIdx.x & 63;
    const int64_t nunits = (a.ngran / a.gsize) * a.nruns;        // instances x runs
    const int64_t nw = (int64_t)gridDim.x * kWaves;
    // (dispatch order here: XCD-contiguous order measured 10 % slower for this kernel)
    for (int64_t u = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); u < nunits; u += nw) {
        const int64_t i = u / a.nruns, k = u - i * a.nruns;
        int64_t po, len, disp;
        if (a.n1) {             // two-level regular layout: run k computed, no tables
            const int64_t k1 = k / a.n1;
            po = k * a.gblen * G;
            len = a.gblen;
            disp = a.first + k1 * a.stride2 + (k - k1 * a.n1) * a.stride;
        } else {
            po = a.poff[k];
            len = (a.poff[k + 1] - po) / G;
            disp = a.disp[k];
        }
        T* t = reinterpret_cast<T*>(a.typed + i * a.extent + disp);
        T* p = reinterpret_cast<T*>(a.packed + i * a.size + po);
        for (int64_t j0 = lane; j0 < len; j0 += 64 * kUnroll) {
            T v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t j = j0 + 64 * u;
                if (j < len) {
                    if constexpr (UNPACK) v[u] = __builtin_nontemporal_load(p + j);
                    else v[u] = t[j];
                }
            }
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const int64_t j = j0 + 64 * u;
                if (j < len) {
                    if constexpr (UNPACK) t[j] = v[u];
                    else __builtin_nontemporal_store(v[u], p + j);
                }
            }
        }
    }
}

// typed element (op)= packed element.  E = element bytes; granules are whole
// elements.  ALIGNED: every element address is a multiple of alignof(T);
// otherwise the element moves through byte copies.
template <int OP, class T, bool ALIGNED>
__device__ __forceinline__ void acc_elem(char* t, const char* p)
{
    constexpr int E = (int)sizeof(T);
    if constexpr (ALIGNED) {
        T* tt = reinterpret_cast<T*>(t);
        *tt = Fn<OP>::apply(*tt, *reinterpret_cast<const T*>(p));
    } else {
        T x, y;
        __builtin_memcpy(&x, t, E);
        __builtin_memcpy(&y, p, E);
        x = Fn<OP>::apply(x, y);
        __builtin_memcpy(t, &x, E);
    }
}

// The derived-target accumulate, in the pack kernels' tile form
// (k_dt_pack_tile): one-wave workgroups in dispatch order, kUnroll x 64
// consecutive elements each, every operand of the tile loaded before the first
// combine when the elements are aligned.  (Rounds 2-5 also carried a
// grid-stride form; the tile form beat it at every size measured, below.)
template <int OP, class T, bool REG, bool ALIGNED>
__global__ __launch_bounds__(64) void k_dt_acc_tile(CopyArgs a)
{
    constexpr int E = (int)sizeof(T);
    const int64_t g0 = (int64_t)blockIdx.x * (64 * kUnroll) + threadIdx.x;
    if constexpr (ALIGNED) {
        T x[kUnroll], y[kUnroll];
        T* tt[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t g = g0 + u * 64;
            if (g < a.ngran) {
                tt[u] = reinterpret_cast<T*>(a.typed + typed_off<E, REG, false>(a, g));
                x[u] = *tt[u];
                y[u] = reinterpret_cast<const T*>(a.packed)[g];
            }
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
            if (g0 + u * 64 < a.ngran) *tt[u] = Fn<OP>::apply(x[u], y[u]);
    } else {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const int64_t g = g0 + u * 64;
            if (g < a.ngran) acc_elem<OP, T, false>(a.typed + typed_off<E, REG, false>(a, g), a.packed + g * E);
        }
    }
}

// ---- host side ---------------------------------------------------------------
int grid_for(int64_t n)
{
    // a few waves of workgroups over 256 CUs; the loops are grid-stride
    const int64_t want = (n + kPackBlock - 1) / kPackBlock;
    return (int)(want < 8192 ? (want > 0 ? want : 1) : 8192);
}

CopyArgs make_args(const DevLayout& L, int64_t count, void* typed, void* packed, int G)
{
    CopyArgs a{};
    a.typed = static_cast<char*>(typed);
    a.packed = static_cast<char*>(packed);
    a.extent = L.extent;
    a.size = L.size;
    a.gsize = L.size / G;
    a.ngran = count * a.gsize;
    a.nruns = L.nruns;
    if (L.regular) {
        a.first = L.first;
        a.stride = L.stride;
        a.gblen = L.blen / G;
        a.n1 = L.n1;
        a.stride2 = L.stride2;
    } else {
        a.disp = L.disp;
        a.poff = L.poff;
        a.nruns = L.nruns;
    }
    a.fd_size = FastDiv((uint32_t)(a.gsize < 0xffffffffll ? a.gsize : 1));
    a.fd_blen = FastDiv((uint32_t)(a.gblen > 0 && a.gblen < 0xffffffffll ? a.gblen : 1));
    a.fd_n1 = FastDiv((uint32_t)(a.n1 > 0 && a.n1 < 0xffffffffll ? a.n1 : 1));
    return a;
}

// Average run length (in granules) from which a wave per run beats the
// per-granule binary search.
constexpr int64_t kRunParallelMin = 8;

}  // namespace dev

// Pack/unpack geometry (msx_tune_pack): 0 = by size (the tile form when the
// call's typed span plus packed bytes exceed pack_tile_min()), 1 = always the
// grid-stride form, 2 = always the tile form.
int g_pack_mode = 0;

constexpr size_t kPackTileMin = (size_t)512 << 20;
size_t pack_tile_min() { return kPackTileMin; }

// A derived-target accumulate always runs k_dt_acc_tile.  Self-targeted fp32
// SUM MPI_Accumulate through a 16-B-block vector target type, grid-stride ->
// tile form, three interleaved rounds (round 3,
// profiles/r03/acc_geometry/): 256 MiB window 144 -> 140 us per call, 1 GiB
// 663 -> 521 us.

int pack_tune_set(int mode)
{
    if (mode < 0 || mode > 2) return -1;
    g_pack_mode = mode;
    return 0;
}

namespace dev {

template <int G, bool UNPACK>
hipError_t run_copy(const CopyArgs& a, bool reg, hipStream_t s)
{
    const bool narrow = a.ngran < (int64_t)0xffffffffll;
    const dim3 block(kPackBlock);
    // Two-level regular layouts (2-D / 3-D subarrays) map granules by two
    // magic-number divisions in the tile form, which beats the wave-per-run
    // kernel at every size measured (3-D fp32 subarray, 1536-B rows, runs ->
    // tile: 256 MiB pack 35.0 -> 34.3 us, unpack 37.7 -> 37.1; 2 GiB pack
    // 348.5 -> 313.5, unpack 378.4 -> 347.4; scripts/pack_size_probe.py,
    // profiles/r03/pack_geometry/).  msx_tune_pack 1 keeps the wave-per-run
    // kernel for them, 2 forces the tile form for every layout.
    const bool two_level = reg && a.n1 != 0;
    const bool tile_first = g_pack_mode == 2 || (g_pack_mode == 0 && two_level);
    // long runs: irregular tables, or a two-level regular layout under mode 1
    if (!tile_first && (!reg || a.n1) && a.gsize >= kRunParallelMin * a.nruns) {
        const int64_t units = (a.ngran / a.gsize) * a.nruns;
        const int64_t want = (units + kPackBlock / 64 - 1) / (kPackBlock / 64);
        const dim3 grid((unsigned)(want < 8192 ? want : 8192));
        hipLaunchKernelGGL((k_dt_runs<G, UNPACK>), grid, block, 0, s, a);
        return hipGetLastError();
    }
    const size_t span = (size_t)(a.ngran / a.gsize) * (size_t)a.extent + (size_t)a.ngran * G;
    if (tile_first || (g_pack_mode == 0 && span > pack_tile_min())) {
        const int64_t want = (a.ngran + 64 * kUnroll - 1) / (64 * kUnroll);
        if (want <= 0x7fffffffll) {
            const dim3 tg((unsigned)want), tb(64);
            if (reg && narrow) hipLaunchKernelGGL((k_dt_pack_tile<G, true, true, UNPACK>), tg, tb, 0, s, a);
            else if (reg) hipLaunchKernelGGL((k_dt_pack_tile<G, true, false, UNPACK>), tg, tb, 0, s, a);
            else hipLaunchKernelGGL((k_dt_pack_tile<G, false, false, UNPACK>), tg, tb, 0, s, a);
            return hipGetLastError();
        }
    }
    const dim3 grid(grid_for(a.ngran));
    if (reg && narrow) hipLaunchKernelGGL((k_dt_pack<G, true, true, UNPACK>), grid, block, 0, s, a);
    else if (reg) hipLaunchKernelGGL((k_dt_pack<G, true, false, UNPACK>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_dt_pack<G, false, false, UNPACK>), grid, block, 0, s, a);
    return hipGetLastError();
}

template <bool UNPACK>
hipError_t copy_g(int G, const CopyArgs& a, bool reg, hipStream_t s)
{
    switch (G) {
    case 16: return run_copy<16, UNPACK>(a, reg, s);
    case 8: return run_copy<8, UNPACK>(a, reg, s);
    case 4: return run_copy<4, UNPACK>(a, reg, s);
    case 2: return run_copy<2, UNPACK>(a, reg, s);
    default: return run_copy<1, UNPACK>(a, reg, s);
    }
}

// Which (op, element) pairs have a kernel: the builtin ops' tables (op.cpp:739-1883).
template <int OP, class T> struct AccLegal {
    static constexpr bool arith = std::is_arithmetic<T>::value;
    static constexpr bool value =
        ((OP == O_MAX || OP == O_MIN || OP == O_LAND || OP == O_LOR || OP == O_LXOR) && arith) ||
        ((OP == O_SUM || OP == O_PROD) && (arith || std::is_same<T, c32>::value || std::is_same<T, c64>::value)) ||
        ((OP == O_BAND || OP == O_BOR || OP == O_BXOR) && std::is_integral<T>::value) ||
        ((OP == O_MAXLOC || OP == O_MINLOC) &&
         (std::is_same<T, loc_ii>::value || std::is_same<T, loc_fi>::value || std::is_same<T, loc_si>::value ||
          std::is_same<T, loc_di>::value || std::is_same<T, loc_ff>::value || std::is_same<T, loc_dd>::value));
};

template <int OP, class T>
hipError_t run_acc(const DevLayout& L, int64_t count, const void* packed, void* typed, hipStream_t s)
{
    if constexpr (!AccLegal<OP, T>::value) {
        return hipErrorInvalidValue;
    } else {
        constexpr int E = (int)sizeof(T);
        // every run offset / length must hold whole elements for the element map
        if (L.size % E) return hipErrorInvalidValue;
        CopyArgs a = make_args(L, count, typed, const_cast<void*>(packed), E);
        if (L.regular && (L.blen % E)) return hipErrorInvalidValue;
        const bool aligned = L.align >= (int)alignof(T);
        const bool reg = L.regular != 0;
        const int64_t tiles = (a.ngran + 64 * kUnroll - 1) / (64 * kUnroll);
        if (tiles == 0) return hipSuccess;
        if (tiles > 0x7fffffffll) return hipErrorInvalidValue;     // > 2^39 elements: beyond any HBM
        const dim3 tg((unsigned)tiles), tb(64);
        if (reg && aligned) hipLaunchKernelGGL((k_dt_acc_tile<OP, T, true, true>), tg, tb, 0, s, a);
        else if (reg) hipLaunchKernelGGL((k_dt_acc_tile<OP, T, true, false>), tg, tb, 0, s, a);
        else if (aligned) hipLaunchKernelGGL((k_dt_acc_tile<OP, T, false, true>), tg, tb, 0, s, a);
        else hipLaunchKernelGGL((k_dt_acc_tile<OP, T, false, false>), tg, tb, 0, s, a);
        return hipGetLastError();
    }
}

template <int OP>
hipError_t acc_kind(Kind k, const DevLayout& L, int64_t count, const void* packed, void* typed, hipStream_t s)
{
    switch (k) {
    case K_I8: return run_acc<OP, int8_t>(L, count, packed, typed, s);
    case K_U8: case K_BOOL: return run_acc<OP, uint8_t>(L, count, packed, typed, s);
    case K_I16: return run_acc<OP, int16_t>(L, count, packed, typed, s);
    case K_U16: return run_acc<OP, uint16_t>(L, count, packed, typed, s);
    case K_I32: return run_acc<OP, int32_t>(L, count, packed, typed, s);
    case K_U32: return run_acc<OP, uint32_t>(L, count, packed, typed, s);
    case K_I64: return run_acc<OP, int64_t>(L, count, packed, typed, s);
    case K_U64: return run_acc<OP, uint64_t>(L, count, packed, typed, s);
    case K_F32: return run_acc<OP, float>(L, count, packed, typed, s);
    case K_F64: return run_acc<OP, double>(L, count, packed, typed, s);
    case K_C32: return run_acc<OP, c32>(L, count, packed, typed, s);
    case K_C64: return run_acc<OP, c64>(L, count, packed, typed, s);
    case K_LOC_II: return run_acc<OP, loc_ii>(L, count, packed, typed, s);
    case K_LOC_FI: return run_acc<OP, loc_fi>(L, count, packed, typed, s);
    case K_LOC_SI: return run_acc<OP, loc_si>(L, count, packed, typed, s);
    case K_LOC_DI: return run_acc<OP, loc_di>(L, count, packed, typed, s);
    case K_LOC_FF: return run_acc<OP, loc_ff>(L, count, packed, typed, s);
    case K_LOC_DD: return run_acc<OP, loc_dd>(L, count, packed, typed, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace dev

hipError_t launch_dt_copy(const DevLayout& L, int64_t count, void* typed, void* packed, bool unpack,
                          hipStream_t s)
{
    if (count <= 0 || L.size == 0) return hipSuccess;
    const int G = L.align;
    if (G < 1 || G > 16 || (G & (G - 1)) || L.size % G || (L.regular && L.blen % G))
        return hipErrorInvalidValue;
    dev::CopyArgs a = dev::make_args(L, count, typed, packed, G);
    return unpack ? dev::copy_g<true>(G, a, L.regular != 0, s) : dev::copy_g<false>(G, a, L.regular != 0, s);
}

hipError_t launch_dt_acc(int opidx, Kind k, const DevLayout& L, int64_t count, const void* packed,
                         void* typed, hipStream_t s)
{
    if (count <= 0 || L.size == 0) return hipSuccess;
    switch (opidx) {
    case O_MAX: return dev::acc_kind<O_MAX>(k, L, count, packed, typed, s);
    case O_MIN: return dev::acc_kind<O_MIN>(k, L, count, packed, typed, s);
    case O_SUM: return dev::acc_kind<O_SUM>(k, L, count, packed, typed, s);
    case O_PROD: return dev::acc_kind<O_PROD>(k, L, count, packed, typed, s);
    case O_LAND: return dev::acc_kind<O_LAND>(k, L, count, packed, typed, s);
    case O_BAND: return dev::acc_kind<O_BAND>(k, L, count, packed, typed, s);
    case O_LOR: return dev::acc_kind<O_LOR>(k, L, count, packed, typed, s);
    case O_BOR: return dev::acc_kind<O_BOR>(k, L, count, packed, typed, s);
    case O_LXOR: return dev::acc_kind<O_LXOR>(k, L, count, packed, typed, s);
    case O_BXOR: return dev::acc_kind<O_BXOR>(k, L, count, packed, typed, s);
    case O_MINLOC: return dev::acc_kind<O_MINLOC>(k, L, count, packed, typed, s);
    case O_MAXLOC: return dev::acc_kind<O_MAXLOC>(k, L, count, packed, typed, s);
    case O_REPLACE: return launch_dt_copy(L, count, typed, const_cast<void*>(packed), true, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace msx
