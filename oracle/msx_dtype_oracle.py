"""msx_dtype_oracle — CPU restatement of MS-MPI's derived-datatype semantics.

ORACLE — TEST INFRASTRUCTURE ONLY; PARITY UNPINNED (no reference test or
output covers datatypes; pinned by the MPI-2.2 worked examples).
Imported by tests/ as the checker of the
datatype engine (microsoft-mpi_amd/csrc/msx_dtype.cpp + msx_pack.hip); the
product never imports it and there is no CPU packing path in the product.

A type is restated the way the MPI standard defines it: a type map, i.e. the
ordered list of (byte displacement, basic element size) pairs of one instance,
plus the attributes the reference computes next to it.  Packing is the plain
gather of those elements (MPID_Segment_pack's result, mpid/segment.cpp), and
unpack / accumulate are the scatter and the per-element combine over the same
list.  This is deliberately NOT the product's representation (merged byte runs
walked by a granule address map on the GPU), so the two are independent.

Attribute formulas follow the reference:
  builtins / pair types      mpid/datatype.cpp:222-306, 1282-1293 (LLP64 sizes)
  MPID_DATATYPE_*_LB_UB      include/datatype.h:522-611
  MPID_Type_vector           mpid/datatype.cpp:2495-2622 (contiguous, hvector)
  MPID_Type_indexed          mpid/datatype.cpp:1870-2060
  MPID_Type_struct           mpid/datatype.cpp:2214-2473 (+ alignsize 2149-2195)
  MPID_Type_create_resized   mpid/datatype.cpp:1417-1493
  MPID_Type_convert_subarray mpid/datatype.cpp:3274-3399
  MPI_Type_create_darray     api/mpi_datatype.cpp:218-600 with MPIR_Type_block /
                             MPIR_Type_cyclic, mpid/datatype.cpp:409-637
Parity pin: no reference test covers datatypes and the
reference's datatype engine does not build here (it needs the CH3 runtime), so
the restatement is pinned by the MPI-2.2 standard's worked examples
(tests/test_dtype_cpu.py::test_oracle_standard_examples, §4.1.2-4.1.4).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

# handles (include/mpi.h values)
MPI_LB = 0x4C000010
MPI_UB = 0x4C000011
PAIR_TYPES = {   # handle: (size1, size2, offset2, extent, alignsize)  datatype.cpp:1282-1293
    0x8C000000: (4, 4, 4, 8, 4),      # MPI_FLOAT_INT
    0x8C000001: (8, 4, 8, 16, 8),     # MPI_DOUBLE_INT
    0x8C000002: (4, 4, 4, 8, 4),      # MPI_LONG_INT (long = 4 B)
    0x8C000003: (2, 4, 4, 8, 4),      # MPI_SHORT_INT
    0x8C000004: (8, 4, 8, 16, 8),     # MPI_LONG_DOUBLE_INT (long double = double)
}
# builtin alignsize exceptions (datatype.cpp:262-287)
_ALIGN4 = {0x4C000816, 0x4C00082A, 0x4C000828, 0x4C00081E, 0x4C000829, 0x4C000843, 0x4C000845}
_ALIGN8 = {0x4C001022, 0x4C001023, 0x4C001024, 0x4C00102A, 0x4C001046, 0x4C001047}


def basic_size(h: int) -> int:
    """Element bytes of a builtin handle: byte 1 (include/datatype.h:36)."""
    return (h >> 8) & 0xFF


@dataclass
class OType:
    typemap: List[Tuple[int, int]] = field(default_factory=list)   # (disp, element bytes)
    size: int = 0
    lb: int = 0
    ub: int = 0
    true_lb: int = 0
    true_ub: int = 0
    sticky_lb: bool = False
    sticky_ub: bool = False
    alignsize: int = 0
    builtin: bool = False
    marker: bool = False          # MPI_LB / MPI_UB

    @property
    def extent(self) -> int:
        return self.ub - self.lb


def predefined(h: int) -> OType:
    if h in PAIR_TYPES:
        s1, s2, off2, ext, al = PAIR_TYPES[h]
        return OType([(0, s1), (off2, s2)], s1 + s2, 0, ext, 0, off2 + s2, alignsize=al)
    s = basic_size(h)
    al = 4 if h in _ALIGN4 else 8 if h in _ALIGN8 else s
    t = OType([(0, s)] if s else [], s, 0, s, 0, s, alignsize=al, builtin=True)
    t.marker = h in (MPI_LB, MPI_UB)
    return t


def _block_lb_ub(cnt, disp, olb, oub, oext):
    if cnt == 0:
        return olb + disp, oub + disp
    if oub >= olb:
        return olb + disp, oub + disp + oext * (cnt - 1)
    return olb + disp + oext * (cnt - 1), oub + disp


def _vector_lb_ub(cnt, stride, blk, olb, oub, oext):
    if cnt == 0 or blk == 0:
        return olb, oub
    if stride >= 0 and oext >= 0:
        return olb, oub + oext * (blk - 1) + stride * (cnt - 1)
    if stride < 0 and oext >= 0:
        return olb + stride * (cnt - 1), oub + oext * (blk - 1)
    if stride >= 0 and oext < 0:
        return olb + oext * (blk - 1), oub + stride * (cnt - 1)
    return olb + oext * (blk - 1) + stride * (cnt - 1), oub


def _zerolen() -> OType:
    return OType()


def hvector(count: int, blen: int, stride_bytes: int, old: OType) -> OType:
    if count == 0:
        return _zerolen()
    t = OType(size=count * blen * old.size, sticky_lb=old.sticky_lb, sticky_ub=old.sticky_ub,
              alignsize=old.alignsize)
    t.lb, t.ub = _vector_lb_ub(count, stride_bytes, blen, old.lb, old.ub, old.extent)
    t.true_lb = t.lb + (old.true_lb - old.lb)
    t.true_ub = t.ub + (old.true_ub - old.ub)
    for j in range(count):
        for b in range(blen):
            base = j * stride_bytes + b * old.extent
            t.typemap += [(base + d, s) for d, s in old.typemap]
    return t


def vector(count, blen, stride, old):
    return hvector(count, blen, stride * old.extent, old)


def contiguous(count, old):
    return hvector(count, 1, old.extent, old)


def hindexed(blens, disps_bytes, old: OType) -> OType:
    live = [i for i, b in enumerate(blens) if b > 0]
    if not live:
        return _zerolen()
    t = OType(sticky_lb=old.sticky_lb, sticky_ub=old.sticky_ub, alignsize=old.alignsize)
    lbs, ubs = zip(*[_block_lb_ub(blens[i], disps_bytes[i], old.lb, old.ub, old.extent) for i in live])
    t.lb, t.ub = min(lbs), max(ubs)
    t.true_lb = t.lb + (old.true_lb - old.lb)
    t.true_ub = t.ub + (old.true_ub - old.ub)
    t.size = sum(blens[i] for i in live) * old.size
    for i, b in enumerate(blens):
        for k in range(b):
            base = disps_bytes[i] + k * old.extent
            t.typemap += [(base + d, s) for d, s in old.typemap]
    return t


def indexed(blens, disps, old):
    return hindexed(blens, [d * old.extent for d in disps], old)


def struct(blens, disps, olds: List[OType]) -> OType:
    if not any(b > 0 for b in blens):
        return _zerolen()
    t = OType()
    slb = sub = tlb = tub = None
    for b, d, o in zip(blens, disps, olds):
        if b == 0:
            continue
        lb, ub = _block_lb_ub(b, d, o.lb, o.ub, o.extent)
        tl, tu = lb + (o.true_lb - o.lb), ub + (o.true_ub - o.ub)
        t.size += o.size * b
        is_lb = o.marker and o is _LB_SENTINEL
        is_ub = o.marker and o is _UB_SENTINEL
        if is_lb or (not o.builtin and o.sticky_lb):
            slb = lb if slb is None else min(slb, lb)
        if is_ub or (not o.builtin and o.sticky_ub):
            sub = ub if sub is None else max(sub, ub)
        if not o.marker:
            tlb = tl if tlb is None else min(tlb, tl)
            tub = tu if tub is None else max(tub, tu)
            for k in range(b):
                base = d + k * o.extent
                t.typemap += [(base + x, s) for x, s in o.typemap]
    t.sticky_lb, t.sticky_ub = slb is not None, sub is not None
    t.true_lb, t.true_ub = tlb or 0, tub or 0
    t.lb = slb if slb is not None else t.true_lb
    t.ub = sub if sub is not None else t.true_ub
    # MPID_Type_struct_alignsize: the largest alignment, reduced to the lowest
    # set bit of a displacement that is not a multiple of it
    al = 0
    for d, o in zip(disps, olds):
        if o.marker or o.alignsize == 0:
            continue
        a = o.alignsize
        if d % a:
            u = d % a
            a = u & -u
        al = max(al, a)
    t.alignsize = al
    if not t.sticky_lb and not t.sticky_ub and al:
        eps = t.extent % al
        if eps:
            t.ub += al - eps
    return t


_LB_SENTINEL = predefined(MPI_LB)
_UB_SENTINEL = predefined(MPI_UB)


def marker(h: int) -> OType:
    return _LB_SENTINEL if h == MPI_LB else _UB_SENTINEL


def resized(old: OType, lb: int, extent: int) -> OType:
    t = OType(list(old.typemap), old.size, lb, lb + extent, old.true_lb, old.true_ub,
              True, True, old.alignsize)
    return t


def subarray(sizes, subsizes, starts, order_c: bool, old: OType) -> OType:
    n = len(sizes)
    ext = old.extent
    if order_c:
        sizes, subsizes, starts = sizes[::-1], subsizes[::-1], starts[::-1]
    # Fortran order from here: dimension 0 fastest
    if n == 1:
        t = contiguous(subsizes[0], old)
    else:
        t = vector(subsizes[1], subsizes[0], sizes[0], old)
        step = sizes[0] * ext
        for i in range(2, n):
            step *= sizes[i - 1]
            t = hvector(subsizes[i], 1, step, t)
    disp, step = starts[0], 1
    for i in range(1, n):
        step *= sizes[i - 1]
        disp += step * starts[i]
    full = ext
    for s in sizes:
        full *= s
    return struct([1, 1, 1], [0, disp * ext, full], [marker(MPI_LB), t, marker(MPI_UB)])


DIST_BLOCK, DIST_CYCLIC, DIST_NONE, DFLT_DARG = 121, 122, 123, -49767


def _dims_after(gsizes, dim, order_c):
    """Product of the faster-varying global sizes (the stride factor)."""
    p = 1
    for i in (range(dim + 1, len(gsizes)) if order_c else range(dim)):
        p *= gsizes[i]
    return p


def _darray_block(gsizes, dim, nprocs, rank, darg, order_c, ext, old):
    g = gsizes[dim]
    blk = (g + nprocs - 1) // nprocs if darg == DFLT_DARG else darg
    mysize = max(0, min(blk, g - blk * rank))
    fastest = dim == len(gsizes) - 1 if order_c else dim == 0
    if fastest:
        t = contiguous(mysize, old)
    else:
        t = hvector(mysize, 1, ext * _dims_after(gsizes, dim, order_c), old)
    return t, (0 if mysize == 0 else blk * rank)


def _darray_cyclic(gsizes, dim, nprocs, rank, darg, order_c, ext, old):
    blk = 1 if darg == DFLT_DARG else darg
    st_i, end_i = rank * blk, gsizes[dim] - 1
    local = 0
    if end_i >= st_i:
        per = nprocs * blk
        local = ((end_i - st_i + 1) // per) * blk + min((end_i - st_i + 1) % per, blk)
    count, rem = divmod(local, blk)
    stride = nprocs * blk * ext * _dims_after(gsizes, dim, order_c)
    t = hvector(count, blk, stride, old)
    if rem:
        t = struct([1, rem], [0, count * stride], [t, old])
    first = dim == len(gsizes) - 1 if order_c else dim == 0
    if first:
        t = struct([1, 1, 1], [0, rank * blk * ext, ext * gsizes[dim]], [marker(MPI_LB), t, marker(MPI_UB)])
        off = 0
    else:
        off = rank * blk
    return t, (0 if local == 0 else off)


def darray(size, rank, gsizes, distribs, dargs, psizes, order_c, old: OType) -> OType:
    n = len(gsizes)
    ext = old.extent
    coords, procs, r = [], size, rank
    for i in range(n):
        procs //= psizes[i]
        coords.append(r // procs)
        r %= procs
    st = [0] * n
    cur = old
    for i in (range(n - 1, -1, -1) if order_c else range(n)):
        if distribs[i] == DIST_CYCLIC:
            cur, st[i] = _darray_cyclic(gsizes, i, psizes[i], coords[i], dargs[i], order_c, ext, cur)
        elif distribs[i] == DIST_BLOCK:
            cur, st[i] = _darray_block(gsizes, i, psizes[i], coords[i], dargs[i], order_c, ext, cur)
        else:
            cur, st[i] = _darray_block(gsizes, i, psizes[i], coords[i], DFLT_DARG, order_c, ext, cur)
    disp, step = 0, 1
    dims = list(range(n - 1, -1, -1)) if order_c else list(range(n))
    for k, i in enumerate(dims):
        if k:
            step *= gsizes[dims[k - 1]]
        disp += step * st[i]
    full = ext
    for g in gsizes:
        full *= g
    return struct([1, 1, 1], [0, disp * ext, full], [marker(MPI_LB), cur, marker(MPI_UB)])


# ---- data movement --------------------------------------------------------------
def pack(t: OType, count: int, typed: np.ndarray, base: int) -> np.ndarray:
    """Gather `count` instances starting at byte `base` of the uint8 array."""
    out = []
    for i in range(count):
        off = base + i * t.extent
        for d, s in t.typemap:
            out.append(typed[off + d: off + d + s])
    return np.concatenate(out) if out else np.zeros(0, np.uint8)


def unpack(t: OType, count: int, packed: np.ndarray, typed: np.ndarray, base: int) -> None:
    p = 0
    for i in range(count):
        off = base + i * t.extent
        for d, s in t.typemap:
            typed[off + d: off + d + s] = packed[p: p + s]
            p += s


def span(t: OType, count: int) -> Tuple[int, int]:
    """Byte range [lo, hi) of `count` instances relative to the buffer address."""
    if not t.typemap or count == 0:
        return 0, 0
    lo = min(d for d, _ in t.typemap)
    hi = max(d + s for d, s in t.typemap)
    shift = (count - 1) * t.extent
    return lo + min(0, shift), hi + max(0, shift)
