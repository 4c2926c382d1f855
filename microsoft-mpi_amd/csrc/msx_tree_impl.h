// msx_tree_impl.h — host-side launch of k_tree (msx_tree_dev.h) for one MPI_Op
// family per translation unit (msx_tree_sum/prod/max/min/loc/land/lor/lxor/
// bit.hip), so the template instantiations compile in parallel.  Included by
// those files only.
#pragma once
#include "msx_tree_dev.h"

namespace msx {
namespace {

using namespace dev;

constexpr int kTreeBlock = 256;
constexpr int kTreeGridCap = 4096;          // generic kernel: grid-stride beyond this
constexpr int kFixedGridCap = 1 << 20;      // compile-time-source kernel: one tile per workgroup

template <int OP, class T, class VT, bool NT = false, int NL = 0, int U = 1, bool CHAIN = false,
          int BLOCK = kTreeBlock, bool MASKED = false>
hipError_t run_tree(const TreeArgs& a, int nsrc, void* out, size_t count, hipStream_t s)
{
    bool ok = ((uintptr_t)out & 15) == 0;
    for (int k = 0; k < nsrc; ++k) ok = ok && a.s[k] && (((uintptr_t)a.s[k] & 15) == 0);
    for (int e = 0; e < a.nextra; ++e) ok = ok && (((uintptr_t)a.extra[e] & 15) == 0);
    constexpr size_t ES = sizeof(T);
    const size_t epv = 16 / ES;
    const size_t nvec = count / epv, tail = count - nvec * epv;
    const size_t work = ok ? (nvec + U - 1) / U + tail : count;
    size_t grid = (work + BLOCK - 1) / BLOCK;
    // one tile per workgroup for the compile-time-source kernel and for the
    // one-wave DRAM-regime form of the generic one; grid-stride beyond
    const size_t cap = (size_t)(NL > 0 || BLOCK == 64 ? kFixedGridCap : kTreeGridCap);
    if (grid > cap) grid = cap;
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL((k_tree<OP, T, VT, BLOCK, NT, NL, U, CHAIN, MASKED>), dim3((unsigned)grid),
                       dim3(BLOCK), 0, s, a, static_cast<T*>(out), nvec, tail, ok ? 1 : 0);
    return hipGetLastError();
}

// The compile-time-source kernel for every tree of up to 8 leaves without
// absent leaves -- full power-of-two trees and non-power-of-two folds (MASKED,
// round 4) -- and every chain of 2-8 sources; the generic kernel for binomial
// trees with absent leaves, p >= 9, and the tuning modes.
// DRAM-regime geometry of the compile-time-source kernel (NT: the sources
// exceed the Infinity Cache): one-wave workgroups in dispatch order, as
// k_combine_dram, so the eight XCDs read neighbouring tiles of every source.
// p = 8 fp32 SUM, uncached sources, two interleaved rounds
// (profiles/r03/tree/dram_geometry/): 64 MiB per
// source 96.3 -> 90.9 us (0.78 -> 0.83 of peak), 128 MiB 201.7 -> 186.8 us
// (0.75 -> 0.81); 64-lane workgroups in XCD-contiguous order and 256-lane ones
// in dispatch order gain 1-2 % only.
template <int OP, class T, class VT, bool NT, int NL, int U, bool CHAIN, bool MASKED = false>
hipError_t run_tree_fixed(const TreeArgs& a, int nsrc, void* out, size_t count, hipStream_t s)
{
    if constexpr (NT) {
        TreeArgs b = a;
        b.xg = -1;
        return run_tree<OP, T, VT, NT, NL, U, CHAIN, 64, MASKED>(b, nsrc, out, count, s);
    }
    return run_tree<OP, T, VT, NT, NL, U, CHAIN, kTreeBlock, MASKED>(a, nsrc, out, count, s);
}

template <int OP, class T, class VT, int U = 1, bool NT = false>
hipError_t run_tree_sel(const TreeArgs& a, int nsrc, void* out, size_t count, hipStream_t s)
{
    if (a.chain) {
        // pairwise exchange chains: p sources (every node size up to 8)
        switch (a.P) {
        case 2: return run_tree_fixed<OP, T, VT, NT, 2, U, true>(a, nsrc, out, count, s);
        case 3: return run_tree_fixed<OP, T, VT, NT, 3, U, true>(a, nsrc, out, count, s);
        case 4: return run_tree_fixed<OP, T, VT, NT, 4, U, true>(a, nsrc, out, count, s);
        case 5: return run_tree_fixed<OP, T, VT, NT, 5, U, true>(a, nsrc, out, count, s);
        case 6: return run_tree_fixed<OP, T, VT, NT, 6, U, true>(a, nsrc, out, count, s);
        case 7: return run_tree_fixed<OP, T, VT, NT, 7, U, true>(a, nsrc, out, count, s);
        case 8: return run_tree_fixed<OP, T, VT, NT, 8, U, true>(a, nsrc, out, count, s);
        default: break;
        }
    } else if (a.pairmask == 0 && a.nleaves == a.P) {
        switch (a.P) {
        case 2: return run_tree_fixed<OP, T, VT, NT, 2, U, false>(a, nsrc, out, count, s);
        case 4: return run_tree_fixed<OP, T, VT, NT, 4, U, false>(a, nsrc, out, count, s);
        case 8: return run_tree_fixed<OP, T, VT, NT, 8, U, false>(a, nsrc, out, count, s);
        default: break;
        }
    } else if (a.nleaves == a.P) {
        // non-power-of-two folds (p = 3, 5, 6, 7: leaf pairs): the leaf count
        // compile-time, the pattern at run time (tree_fixed MASKED).  Binomial
        // trees with ABSENT leaves keep the generic kernel: the masked form
        // loads leaf 0's vectors again for them, which at DRAM sizes costs
        // more than the generic kernel's leaf tests (p = 5/6/7 over 8 leaves,
        // 128 MiB per source: 185/199/215 us masked vs 141/163/179 us generic,
        // profiles/r04/tree_fold_probe.log)
        switch (a.P) {
        case 2: return run_tree_fixed<OP, T, VT, NT, 2, U, false, true>(a, nsrc, out, count, s);
        case 4: return run_tree_fixed<OP, T, VT, NT, 4, U, false, true>(a, nsrc, out, count, s);
        case 8: return run_tree_fixed<OP, T, VT, NT, 8, U, false, true>(a, nsrc, out, count, s);
        default: break;
        }
    }
    if constexpr (NT) {
        // the generic kernel in the same DRAM-regime geometry (run_tree_fixed)
        TreeArgs b = a;
        b.xg = -1;
        return run_tree<OP, T, VT, NT, 0, 1, false, 64>(b, nsrc, out, count, s);
    }
    return run_tree<OP, T, VT, NT>(a, nsrc, out, count, s);
}

// Source loads: plain while the call's sources fit the 256 MiB Infinity Cache
// (just written by the scatter, so partly resident: plain loads hit it),
// non-temporal beyond (streaming: the cache only churns); kTreeNtMin.

template <int OP, class T, class VT, int U = 1>
hipError_t run_tree_auto(const TreeArgs& a, int nsrc, void* out, size_t count, hipStream_t s)
{
    // sources actually read: a tree's leaves plus the second operand of each
    // folded pair (nsrc counts the 2P slots), a chain's P vectors
    const size_t nread = a.chain ? (size_t)a.P : (size_t)a.nleaves + (size_t)__builtin_popcount(a.pairmask);
    if (count * sizeof(T) * nread > kTreeNtMin)
        return run_tree_sel<OP, T, VT, U, true>(a, nsrc, out, count, s);
    return run_tree_sel<OP, T, VT, U, false>(a, nsrc, out, count, s);
}

template <int OP>
hipError_t tree_arith(Kind k, const TreeArgs& a, int ns, void* out, size_t n, hipStream_t s)
{
    switch (k) {
    case K_I8:  return run_tree_auto<OP, int8_t, int8_t>(a, ns, out, n, s);
    case K_U8:  return run_tree_auto<OP, uint8_t, uint8_t>(a, ns, out, n, s);
    case K_I16: return run_tree_auto<OP, int16_t, int16_t>(a, ns, out, n, s);
    case K_U16: return run_tree_auto<OP, uint16_t, uint16_t>(a, ns, out, n, s);
    case K_I32: return run_tree_auto<OP, int32_t, int32_t>(a, ns, out, n, s);
    case K_U32: return run_tree_auto<OP, uint32_t, uint32_t>(a, ns, out, n, s);
    case K_I64: return run_tree_auto<OP, int64_t, int64_t>(a, ns, out, n, s);
    case K_U64: return run_tree_auto<OP, uint64_t, uint64_t>(a, ns, out, n, s);
    case K_F32: return run_tree_auto<OP, float, float>(a, ns, out, n, s);
    case K_F64: return run_tree_auto<OP, double, double>(a, ns, out, n, s);
    default: break;
    }
    if constexpr (OP == O_SUM || OP == O_PROD) {
        if (k == K_C32) return run_tree_auto<OP, c32, c32>(a, ns, out, n, s);
        if (k == K_C64) return run_tree_auto<OP, c64, c64>(a, ns, out, n, s);
    }
    if constexpr (OP == O_LAND || OP == O_LOR || OP == O_LXOR) {
        if (k == K_BOOL) return run_tree_auto<OP, uint8_t, uint8_t>(a, ns, out, n, s);
    }
    return hipErrorInvalidValue;
}

template <int OP>
hipError_t tree_loc(Kind k, const TreeArgs& a, int ns, void* out, size_t n, hipStream_t s)
{
    switch (k) {
    case K_LOC_II: return run_tree_auto<OP, loc_ii, loc_ii>(a, ns, out, n, s);
    case K_LOC_FI: return run_tree_auto<OP, loc_fi, loc_fi>(a, ns, out, n, s);
    case K_LOC_SI: return run_tree_auto<OP, loc_si, loc_si>(a, ns, out, n, s);
    case K_LOC_DI: return run_tree_auto<OP, loc_di, loc_di>(a, ns, out, n, s);
    case K_LOC_FF: return run_tree_auto<OP, loc_ff, loc_ff>(a, ns, out, n, s);
    case K_LOC_DD: return run_tree_auto<OP, loc_dd, loc_dd>(a, ns, out, n, s);
    default: return hipErrorInvalidValue;
    }
}

}  // namespace

template <int OP>
hipError_t tree_dispatch(Kind k, const TreeArgs& a, int ns, void* out, size_t n, hipStream_t s)
{
    if constexpr (OP == O_BAND || OP == O_BOR || OP == O_BXOR)     // raw bytes on 32-bit lanes
        return run_tree_auto<OP, uint8_t, uint32_t>(a, ns, out, n * kind_size(k), s);
    else if constexpr (OP == O_MAXLOC || OP == O_MINLOC)
        return tree_loc<OP>(k, a, ns, out, n, s);
    else
        return tree_arith<OP>(k, a, ns, out, n, s);
}

}  // namespace msx
