// msx_dev_ops.h — device element types and op functors shared by the gfx950
// kernels: msx_kernels.hip (contiguous combine, collective trees) and
// msx_pack.hip (datatype pack / unpack and the non-contiguous accumulate).
//
// Element semantics follow src/mpi/msmpi/mpid/op.cpp:14-340 (cited at each
// functor).  Every translation unit that includes this is compiled with
// -ffp-contract=off and IEEE denormals.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

#include "msx_types.h"

namespace msx {
namespace dev {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ---- element types (layouts of op.cpp:280-340, padding made explicit so a
// struct assignment copies every byte like the reference's `*this = rhs`) ----
struct c32 { float re, im; };
struct c64 { double re, im; };
struct loc_ii { int32_t v; int32_t l; };
struct loc_fi { float v; int32_t l; };
struct loc_si { int16_t v; int16_t pad; int32_t l; };
struct loc_di { double v; int32_t l; int32_t pad; };
struct loc_ff { float v; float l; };
struct loc_dd { double v; double l; };
static_assert(sizeof(loc_si) == 8 && sizeof(loc_di) == 16, "loc layout");

// ---- integer arithmetic with two's-complement wrap (MSVC semantics) -------
template <class T> struct Wrap {
    using U = typename std::make_unsigned<T>::type;
    using W = typename std::conditional<(sizeof(T) < 4), uint32_t, U>::type;
    __device__ static T add(T a, T b) { return (T)(U)((W)(U)a + (W)(U)b); }
    __device__ static T mul(T a, T b) { return (T)(U)((W)(U)a * (W)(U)b); }
};

// ---- op functors: apply(inout, in) -> new inout ---------------------------
template <int OP> struct Fn;

// Op<T>::Max/Min (op.cpp:18-40): minwindef.h max(inout,in) = inout>in?inout:in
template <> struct Fn<O_MAX> {
    template <class T> __device__ static T apply(T io, T in) { return io > in ? io : in; }
};
template <> struct Fn<O_MIN> {
    template <class T> __device__ static T apply(T io, T in) { return io < in ? io : in; }
};

// ---- floating-point arithmetic with the reference platform's NaN rule ------
// IEEE 754 leaves a NaN result's payload open.  The reference runs on x86-64
// SSE: `x op y` yields x's NaN (quieted) if x is a NaN, else y's (quieted),
// else the x86 default NaN (sign set) for invalid operations such as inf-inf.
// The kernels apply that rule explicitly with the operands in op.cpp's
// textual order, so NaN results are bit-identical too (oracle: msx_oracle.c).
// Non-NaN results are the plain IEEE op; the check is one compare + select.
__device__ __forceinline__ float qnan(float x) { return __uint_as_float(__float_as_uint(x) | 0x00400000u); }
__device__ __forceinline__ double qnan(double x)
{
    return __longlong_as_double(__double_as_longlong(x) | 0x0008000000000000ll);
}
__device__ __forceinline__ float dnan(float) { return __uint_as_float(0xFFC00000u); }
__device__ __forceinline__ double dnan(double) { return __longlong_as_double((long long)0xFFF8000000000000ull); }
template <class T> __device__ __forceinline__ T x86nan(T r, T x, T y)
{
    if (__builtin_expect(r == r, 1)) return r;
    return (x != x) ? qnan(x) : ((y != y) ? qnan(y) : dnan(x));
}
template <class T> __device__ __forceinline__ T fadd(T x, T y) { return x86nan<T>(x + y, x, y); }
template <class T> __device__ __forceinline__ T fsub(T x, T y) { return x86nan<T>(x - y, x, y); }
template <class T> __device__ __forceinline__ T fmul(T x, T y) { return x86nan<T>(x * y, x, y); }

// Op<T>::Sum (op.cpp:42-52) and complex += (op.cpp:287-292)
template <> struct Fn<O_SUM> {
    template <class T>
    __device__ static typename std::enable_if<std::is_integral<T>::value, T>::type apply(T io, T in)
    { return Wrap<T>::add(io, in); }
    __device__ static float apply(float io, float in) { return fadd(io, in); }
    __device__ static double apply(double io, double in) { return fadd(io, in); }
    __device__ static c32 apply(c32 io, c32 in) { return c32{fadd(io.re, in.re), fadd(io.im, in.im)}; }
    __device__ static c64 apply(c64 io, c64 in) { return c64{fadd(io.re, in.re), fadd(io.im, in.im)}; }
};

// Op<T>::Prod (op.cpp:54-64) and complex *= (op.cpp:294-303): 4 mul + 2 add,
// each rounded (no FMA contraction).
template <class C> __device__ inline C cmul(C io, C in)
{
#pragma clang fp contract(off)
    auto r = fsub(fmul(io.re, in.re), fmul(io.im, in.im));
    auto i = fadd(fmul(io.re, in.im), fmul(in.re, io.im));
    return C{r, i};
}
template <> struct Fn<O_PROD> {
    template <class T>
    __device__ static typename std::enable_if<std::is_integral<T>::value, T>::type apply(T io, T in)
    { return Wrap<T>::mul(io, in); }
    __device__ static float apply(float io, float in) { return fmul(io, in); }
    __device__ static double apply(double io, double in) { return fmul(io, in); }
    __device__ static c32 apply(c32 io, c32 in) { return cmul(io, in); }
    __device__ static c64 apply(c64 io, c64 in) { return cmul(io, in); }
};

// Op<T>::LogicalAnd/Or/Xor (op.cpp:66-124): C truthiness, stored as T(0/1).
template <> struct Fn<O_LAND> {
    template <class T> __device__ static T apply(T io, T in)
    { return (T)((io != (T)0) && (in != (T)0)); }
};
template <> struct Fn<O_LOR> {
    template <class T> __device__ static T apply(T io, T in)
    { return (T)((io != (T)0) || (in != (T)0)); }
};
template <> struct Fn<O_LXOR> {
    template <class T> __device__ static T apply(T io, T in)
    {
        bool a = io != (T)0, b = in != (T)0;
        return (T)((a && !b) || (!a && b));
    }
};

// Op<T>::Bitwise* (op.cpp:78-136): byte-independent, so they run on raw words.
template <> struct Fn<O_BAND> {
    template <class T> __device__ static T apply(T io, T in) { return (T)(io & in); }
};
template <> struct Fn<O_BOR> {
    template <class T> __device__ static T apply(T io, T in) { return (T)(io | in); }
};
template <> struct Fn<O_BXOR> {
    template <class T> __device__ static T apply(T io, T in) { return (T)(io ^ in); }
};

// loctype<V,L>::MaxLoc/MinLoc (op.cpp:315-339)
template <> struct Fn<O_MAXLOC> {
    template <class T> __device__ static T apply(T io, T in)
    {
        if (io.v == in.v) { io.l = io.l < in.l ? io.l : in.l; return io; }
        return (io.v < in.v) ? in : io;
    }
};
template <> struct Fn<O_MINLOC> {
    template <class T> __device__ static T apply(T io, T in)
    {
        if (io.v == in.v) { io.l = io.l < in.l ? io.l : in.l; return io; }
        return (io.v > in.v) ? in : io;
    }
};

// ---- 16-byte vector apply ------------------------------------------------------
template <int OP, class VT>
__device__ __forceinline__ u32x4 apply_vec(u32x4 io, u32x4 in)
{
    constexpr int N = 16 / (int)sizeof(VT);
    VT a[N], b[N];
    __builtin_memcpy(a, &io, 16);
    __builtin_memcpy(b, &in, 16);
#pragma unroll
    for (int j = 0; j < N; ++j) a[j] = Fn<OP>::apply(a[j], b[j]);
    u32x4 r;
    __builtin_memcpy(&r, a, 16);
    return r;
}

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// XCD-contiguous tile order (the default): workgroup b is dispatched to XCD
// b % 8, so with XCD set XCD x processes one contiguous 1/8 of the tiles (its
// own L2 and a sequential DRAM page stream) instead of every 8th tile.
// Measured on the 256 MiB fp32 SUM: 7.14 TB/s vs 7.01 TB/s in dispatch order
// (interleaved sweep, profiles/r01/bench_sweep.log).
__device__ __forceinline__ unsigned xcd_tile(unsigned b, unsigned nb)
{
    const unsigned q = nb >> 3, r = nb & 7, x = b & 7, j = b >> 3;
    return x * q + (x < r ? x : r) + j;
}

}  // namespace dev
}  // namespace msx
