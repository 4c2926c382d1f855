// msx_combine_dev.h — the streaming combine body `inout[i] = op(inout[i], in[i])`
// (src/mpi/msmpi/mpid/op.cpp:14-160 as an HBM stream).  Device code only;
// included by msx_kernels.hip (the product kernels) and by the bench-only
// probe library (probe/msx_probe.hip), which times the same body under other
// symbols and in other tile orders.
#pragma once

#include "msx_dev_ops.h"

namespace msx {
namespace dev {

// Both registers are inputs of one (empty) asm statement: their loads are
// issued back to back and waited for together, and no use of either can be
// scheduled between them.
__device__ __forceinline__ void issued_together(u32x4& x, u32x4& y)
{
    asm volatile("" : "+v"(x), "+v"(y));
    __builtin_amdgcn_sched_barrier(0);
}

// Tile order: 0 XCD-contiguous eighths, -1 dispatch order (round-robin over
// XCDs), G > 0 XCD x owns interleaved runs of G consecutive tiles.
template <int XG>
__device__ __forceinline__ size_t combine_tile(unsigned b, unsigned nb)
{
    if constexpr (XG == 0) {
        return xcd_tile(b, nb);
    } else if constexpr (XG < 0) {
        return b;
    } else {
        const unsigned full = (nb / (8u * XG)) * (8u * XG);
        if (b >= full) return b;
        const unsigned x = b & 7, j = b >> 3;
        return ((size_t)(j / XG) * 8 + x) * XG + (j % XG);
    }
}

// Elements [0, head) and [head + nvec*EPV, head + nvec*EPV + tail) are scalar;
// the vector body starts at element `head`, 16-byte aligned for both operands.
// T  = element type used for scalar elements;
// VT = lane type used inside a 16-byte vector (== T except bitwise ops, which
//      run on 32-bit words regardless of the MPI element type).
template <int OP, class T, class VT, int UNROLL, int BLOCK, bool NTLD, bool NTST, int XG = 0>
__device__ __forceinline__ void combine_body(const T* __restrict__ in, T* __restrict__ io, size_t head,
                                             size_t nvec, size_t tail)
{
    constexpr size_t EPV = 16 / sizeof(T);
    constexpr size_t TILE = (size_t)BLOCK * UNROLL;
    const u32x4* __restrict__ vin = reinterpret_cast<const u32x4*>(in + head);
    u32x4* __restrict__ vio = reinterpret_cast<u32x4*>(io + head);
    const size_t bid = combine_tile<XG>(blockIdx.x, gridDim.x);

    for (size_t t0 = bid * TILE; t0 < nvec; t0 += (size_t)gridDim.x * TILE) {
        const size_t i0 = t0 + threadIdx.x;
        if (t0 + TILE <= nvec) {
            u32x4 a[UNROLL], b[UNROLL];
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                a[u] = ld<NTLD>(vin + i0 + (size_t)u * BLOCK);
                b[u] = ld<NTLD>(vio + i0 + (size_t)u * BLOCK);
            }
            // Every load of the tile is issued before the first use: without
            // this the compiler hoists work on the first operand (logical ops,
            // complex, byte types) above the second load behind an
            // s_waitcnt vmcnt(0), halving the bytes in flight (-7..10 %).
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) issued_together(a[u], b[u]);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u)
                st<NTST>(vio + i0 + (size_t)u * BLOCK, apply_vec<OP, VT>(b[u], a[u]));
        } else {
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                const size_t i = i0 + (size_t)u * BLOCK;
                if (i < nvec) {
                    u32x4 x = vin[i], y = vio[i];
                    issued_together(x, y);
                    vio[i] = apply_vec<OP, VT>(y, x);
                }
            }
        }
    }

    const size_t nscalar = head + tail;
    if (nscalar) {
        const size_t body_end = head + nvec * EPV;
        for (size_t s = (size_t)blockIdx.x * BLOCK + threadIdx.x; s < nscalar;
             s += (size_t)gridDim.x * BLOCK) {
            const size_t e = s < head ? s : body_end + (s - head);
            io[e] = Fn<OP>::apply(io[e], in[e]);
        }
    }
}

// Operand split of the vector body: head scalars up to 16-byte alignment,
// whole 16-byte vectors, tail scalars.  Operands whose alignments disagree
// (or 16-byte elements off 16-byte alignment) are all-scalar here; the
// realigning kernel takes most of those (msx_kernels.hip, split_shift).
template <class T>
__host__ inline void combine_split(const void* in, const void* io, size_t count, size_t& head, size_t& nvec,
                                   size_t& tail)
{
    constexpr size_t ES = sizeof(T);
    const uintptr_t a = (uintptr_t)in, b = (uintptr_t)io;
    if ((a & 15) != (b & 15) || (a % ES) != 0 || (b % ES) != 0 || (ES == 16 && (a & 15))) {
        head = count; nvec = 0; tail = 0;
        return;
    }
    size_t h = ((16 - (a & 15)) & 15) / ES;
    if (h > count) h = count;
    const size_t rest = count - h;
    const size_t epv = 16 / ES;
    head = h; nvec = rest / epv; tail = rest - nvec * epv;
}

}  // namespace dev
}  // namespace msx
