/*
 * msx_oracle.c — CPU restatement of MS-MPI's element-wise MPI_Op kernels.
 *
 * ORACLE — TEST INFRASTRUCTURE ONLY (see msx_oracle.h).  Plain C, scalar loops,
 * compiled with -ffp-contract=off so floating-point expressions round exactly
 * as written in the reference (no fused multiply-add), like MSVC /fp:precise.
 *
 * Everything below restates /root/reference/src/mpi/msmpi/mpid/op.cpp:
 *   Op<T>::Max/Min            op.cpp:18-40   Windows minwindef.h max()/min() macros
 *   Op<T>::Sum/Prod           op.cpp:42-64   integer wrap (MSVC two's complement)
 *   Op<T>::Logical*           op.cpp:66-124  C truthiness, stored back as T(0/1)
 *   Op<T>::Bitwise*           op.cpp:78-136
 *   Op<T>::MaxLoc/MinLoc      op.cpp:138-160 + loctype<V,L> op.cpp:310-340
 *   complex<T> += / *=        op.cpp:280-303 (4 mul + 2 add/sub, no FMA)
 *   CASE_MPI_* type map       op.cpp:343-536 with the LLP64 widths of mpi.h
 *   *_check_dtype tables      op.cpp:739-1883 (USE_STRICT_MPI undefined)
 * The reference loops run backwards (while(--len >= 0)); every element is
 * independent so the direction does not change any result.
 *
 * PARITY UNPINNED (in this task's terms): the reference holds no tests or
 * fixtures for this path and cannot be built here without stand-ins for the
 * Windows headers; the known answers it is checked against
 * (tests/golden/survey_kat.json) came from a shim build.  Independent anchors:
 * x86 SSE silicon for the float / NaN rules (tests/test_x86_nan_rule.py).
 */
#include "msx_oracle.h"

#include <pthread.h>
#include <stdbool.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* datatype -> element class (op.cpp:343-536; mpi.h:284-368)                */
/* ------------------------------------------------------------------------ */
int oracle_kind_of(MPI_Datatype dt)
{
    switch (dt) {
    /* CASE_MPI_C_INTS op.cpp:343-398 (long/unsigned long are 32-bit on Win64) */
    case MPI_INT: case MPI_LONG: case MPI_INT32_T:       return ORK_I32;
    case MPI_UNSIGNED: case MPI_UNSIGNED_LONG: case MPI_UINT32_T: return ORK_U32;
    case MPI_SHORT: case MPI_INT16_T:                     return ORK_I16;
    case MPI_UNSIGNED_SHORT: case MPI_UINT16_T:           return ORK_U16;
    case MPI_LONG_LONG: case MPI_INT64_T:                 return ORK_I64;
    case MPI_UNSIGNED_LONG_LONG: case MPI_UINT64_T:       return ORK_U64;
    case MPI_SIGNED_CHAR: case MPI_INT8_T:                return ORK_I8;
    case MPI_UNSIGNED_CHAR: case MPI_UINT8_T:             return ORK_U8;
    /* CASE_MPI_F_INTS op.cpp:410-434 */
    case MPI_INTEGER: case MPI_INTEGER4:                  return ORK_I32;
    case MPI_AINT: case MPI_OFFSET: case MPI_INTEGER8:    return ORK_I64;
    case MPI_INTEGER1:                                    return ORK_I8;
    case MPI_INTEGER2:                                    return ORK_I16;
    /* CASE_MPI_FLOATS op.cpp:454-469 (long double == double under MSVC) */
    case MPI_FLOAT: case MPI_REAL: case MPI_REAL4:        return ORK_F32;
    case MPI_DOUBLE: case MPI_DOUBLE_PRECISION: case MPI_REAL8:
    case MPI_LONG_DOUBLE:                                 return ORK_F64;
    /* CASE_MPI_COMPLEXES op.cpp:481-495 */
    case MPI_COMPLEX8: case MPI_COMPLEX: case MPI_C_COMPLEX:
    case MPI_C_FLOAT_COMPLEX:                             return ORK_C32;
    case MPI_COMPLEX16: case MPI_DOUBLE_COMPLEX: case MPI_C_DOUBLE_COMPLEX:
    case MPI_C_LONG_DOUBLE_COMPLEX:                       return ORK_C64;
    /* CASE_MPI_LOGICALS op.cpp:498-504: LOGICAL is MPI_Fint */
    case MPI_LOGICAL:                                     return ORK_I32;
    case MPI_C_BOOL:                                      return ORK_BOOL;
    /* CASE_MPI_PRINTABLE_CHARS op.cpp:507-511: MSVC char is signed */
    case MPI_CHAR: case MPI_CHARACTER:                    return ORK_I8;
    /* MPI_BYTE op.cpp:718 (bitwise ops only) */
    case MPI_BYTE:                                        return ORK_U8;
    /* CASE_MPI_LOCTYPES op.cpp:514-536 */
    case MPI_2INT: case MPI_2INTEGER: case MPI_LONG_INT:  return ORK_LOC_II;
    case MPI_FLOAT_INT:                                   return ORK_LOC_FI;
    case MPI_SHORT_INT:                                   return ORK_LOC_SI;
    case MPI_DOUBLE_INT: case MPI_LONG_DOUBLE_INT:        return ORK_LOC_DI;
    case MPI_2REAL:                                       return ORK_LOC_FF;
    case MPI_2DOUBLE_PRECISION:                           return ORK_LOC_DD;
    default:                                              return ORK_NONE;
    }
}

/* loctype<V,L> layouts (op.cpp:310-313): natural C struct layout */
typedef struct { int32_t v; int32_t l; } loc_ii;
typedef struct { float   v; int32_t l; } loc_fi;
typedef struct { int16_t v; int32_t l; } loc_si;   /* 2 B padding */
typedef struct { double  v; int32_t l; } loc_di;   /* 4 B tail padding */
typedef struct { float   v; float   l; } loc_ff;
typedef struct { double  v; double  l; } loc_dd;
typedef struct { float  re, im; } cplx_f;
typedef struct { double re, im; } cplx_d;

int oracle_kind_size(int kind)
{
    switch (kind) {
    case ORK_I8: case ORK_U8: case ORK_BOOL: return 1;
    case ORK_I16: case ORK_U16:              return 2;
    case ORK_I32: case ORK_U32: case ORK_F32: return 4;
    case ORK_I64: case ORK_U64: case ORK_F64: return 8;
    case ORK_C32:    return (int)sizeof(cplx_f);
    case ORK_C64:    return (int)sizeof(cplx_d);
    case ORK_LOC_II: return (int)sizeof(loc_ii);
    case ORK_LOC_FI: return (int)sizeof(loc_fi);
    case ORK_LOC_SI: return (int)sizeof(loc_si);
    case ORK_LOC_DI: return (int)sizeof(loc_di);
    case ORK_LOC_FF: return (int)sizeof(loc_ff);
    case ORK_LOC_DD: return (int)sizeof(loc_dd);
    default: return 0;
    }
}

/* MPI_Type_size of a reducible predefined type.  The pair types are built by
 * SetTypeCharacteristics<T1,T2> (mpid/datatype.cpp:1282-1293): size =
 * sizeof(T1) + sizeof(T2), extent = sizeof(struct {T1 a; T2 b;}).  So
 * DOUBLE_INT / LONG_DOUBLE_INT carry 12 data bytes in a 16-byte extent and
 * SHORT_INT 6 in 8; every other type has size == extent == oracle_kind_size. */
int oracle_type_size(MPI_Datatype dt)
{
    switch (oracle_kind_of(dt)) {
    case ORK_LOC_SI: return (int)(sizeof(int16_t) + sizeof(int32_t));
    case ORK_LOC_DI: return (int)(sizeof(double) + sizeof(int32_t));
    default: return oracle_kind_size(oracle_kind_of(dt));
    }
}

/* ------------------------------------------------------------------------ */
/* legality (op.cpp:739-1883, USE_STRICT_MPI undefined)                      */
/* ------------------------------------------------------------------------ */
enum { G_CINT = 1, G_FINT = 2, G_FLOAT = 4, G_COMPLEX = 8, G_LOGICAL = 16,
       G_CBOOL = 32, G_BYTE = 64, G_PCHAR = 128, G_LOC = 256 };

static int group_of(MPI_Datatype dt)
{
    switch (dt) {
    case MPI_INT: case MPI_LONG: case MPI_SHORT: case MPI_UNSIGNED_SHORT:
    case MPI_UNSIGNED: case MPI_UNSIGNED_LONG: case MPI_LONG_LONG:
    case MPI_UNSIGNED_LONG_LONG: case MPI_SIGNED_CHAR: case MPI_UNSIGNED_CHAR:
    case MPI_INT8_T: case MPI_INT16_T: case MPI_INT32_T: case MPI_INT64_T:
    case MPI_UINT8_T: case MPI_UINT16_T: case MPI_UINT32_T: case MPI_UINT64_T:
        return G_CINT;
    case MPI_INTEGER: case MPI_AINT: case MPI_OFFSET: case MPI_INTEGER1:
    case MPI_INTEGER2: case MPI_INTEGER4: case MPI_INTEGER8:
        return G_FINT;
    case MPI_FLOAT: case MPI_DOUBLE: case MPI_REAL: case MPI_DOUBLE_PRECISION:
    case MPI_LONG_DOUBLE: case MPI_REAL4: case MPI_REAL8:
        return G_FLOAT;
    case MPI_COMPLEX: case MPI_C_COMPLEX: case MPI_C_FLOAT_COMPLEX:
    case MPI_C_DOUBLE_COMPLEX: case MPI_C_LONG_DOUBLE_COMPLEX:
    case MPI_DOUBLE_COMPLEX: case MPI_COMPLEX8: case MPI_COMPLEX16:
        return G_COMPLEX;
    case MPI_LOGICAL:   return G_LOGICAL;
    case MPI_C_BOOL:    return G_CBOOL;
    case MPI_BYTE:      return G_BYTE;
    case MPI_CHAR: case MPI_CHARACTER: return G_PCHAR;
    case MPI_2INT: case MPI_FLOAT_INT: case MPI_LONG_INT: case MPI_SHORT_INT:
    case MPI_DOUBLE_INT: case MPI_LONG_DOUBLE_INT: case MPI_2INTEGER:
    case MPI_2REAL: case MPI_2DOUBLE_PRECISION:
        return G_LOC;
    default: return 0;
    }
}

static int legal_groups(MPI_Op op)
{
    switch (op) {
    case MPI_MAX: case MPI_MIN:                       /* op.cpp:1449-1521 */
        return G_CINT | G_FINT | G_FLOAT | G_PCHAR;
    case MPI_SUM: case MPI_PROD:                      /* op.cpp:1680-1883 */
        return G_CINT | G_FINT | G_FLOAT | G_COMPLEX | G_PCHAR;
    case MPI_LAND: case MPI_LOR: case MPI_LXOR:       /* op.cpp:1026-1386 */
        return G_CINT | G_FINT | G_LOGICAL | G_CBOOL | G_FLOAT | G_PCHAR;
    case MPI_BAND: case MPI_BOR: case MPI_BXOR:       /* op.cpp:739-1002 */
        return G_CINT | G_FINT | G_BYTE | G_LOGICAL | G_PCHAR;
    case MPI_MAXLOC: case MPI_MINLOC:                 /* op.cpp:1543-1571 */
        return G_LOC;
    default:
        return 0;
    }
}

int oracle_op_check(MPI_Op op, MPI_Datatype dt)
{
    int g = group_of(dt);
    return (g != 0 && (legal_groups(op) & g)) ? MPI_SUCCESS : MPI_ERR_OP;
}

/* ------------------------------------------------------------------------ */
/* element loops                                                             */
/* ------------------------------------------------------------------------ */
/* minwindef.h: #define max(a,b) (((a) > (b)) ? (a) : (b)); min with '<'.
 * Called as max(inout, in) (op.cpp:26,38), so `in` wins on ties and NaN. */
#define WMAX(a, b) (((a) > (b)) ? (a) : (b))
#define WMIN(a, b) (((a) < (b)) ? (a) : (b))

#define LOOP(T, EXPR)                                                        \
    do {                                                                     \
        const T* a = (const T*)in;                                           \
        T* b = (T*)inout;                                                    \
        for (int64_t i = count - 1; i >= 0; --i) { EXPR; }                   \
    } while (0)

/* integer add/mul with MSVC's two's-complement wrap, computed in unsigned so
 * the C restatement has no signed-overflow UB (op.cpp:42-64). */
#define IWRAP_ADD(T, UT) LOOP(T, b[i] = (T)(UT)((UT)b[i] + (UT)a[i]))
#define IWRAP_MUL(T, UT) LOOP(T, b[i] = (T)(UT)((UT)b[i] * (UT)a[i]))

#define INT_KINDS(X)                                                         \
    X(ORK_I8, int8_t, uint32_t) X(ORK_U8, uint8_t, uint32_t)                 \
    X(ORK_I16, int16_t, uint32_t) X(ORK_U16, uint16_t, uint32_t)             \
    X(ORK_I32, int32_t, uint32_t) X(ORK_U32, uint32_t, uint32_t)             \
    X(ORK_I64, int64_t, uint64_t) X(ORK_U64, uint64_t, uint64_t)

static int do_max(int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T, UT) case K: LOOP(T, b[i] = WMAX(b[i], a[i])); return 0;
    INT_KINDS(X)
#undef X
    case ORK_F32: LOOP(float, b[i] = WMAX(b[i], a[i])); return 0;
    case ORK_F64: LOOP(double, b[i] = WMAX(b[i], a[i])); return 0;
    default: return MPI_ERR_OP;
    }
}

static int do_min(int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T, UT) case K: LOOP(T, b[i] = WMIN(b[i], a[i])); return 0;
    INT_KINDS(X)
#undef X
    case ORK_F32: LOOP(float, b[i] = WMIN(b[i], a[i])); return 0;
    case ORK_F64: LOOP(double, b[i] = WMIN(b[i], a[i])); return 0;
    default: return MPI_ERR_OP;
    }
}

/* Floating-point arithmetic with the reference platform's NaN rule.
 * IEEE 754 leaves the payload of a NaN result open; the reference runs on
 * x86-64 SSE, where `x op y` returns x's NaN (quieted) if x is a NaN, else
 * y's NaN (quieted), and the "default NaN" (sign set: 0xFFC00000 /
 * 0xFFF8000000000000) for an invalid operation on non-NaN operands (inf-inf,
 * 0*inf).  The first operand is the one written first in op.cpp:
 * `inout += in` / `inout *= in` (op.cpp:49, 61) and the complex expressions
 * of op.cpp:289-300.  Every non-NaN result is the plain IEEE result. */
static inline float qnan_f(float x) { uint32_t u; memcpy(&u, &x, 4); u |= 0x00400000u; memcpy(&x, &u, 4); return x; }
static inline double qnan_d(double x) { uint64_t u; memcpy(&u, &x, 8); u |= 0x0008000000000000ull; memcpy(&x, &u, 8); return x; }
static inline float dnan_f(void) { uint32_t u = 0xFFC00000u; float x; memcpy(&x, &u, 4); return x; }
static inline double dnan_d(void) { uint64_t u = 0xFFF8000000000000ull; double x; memcpy(&x, &u, 8); return x; }
#define X86_OP(NAME, T, OPER, Q, D)                                          \
    static inline T NAME(T x, T y)                                           \
    {                                                                        \
        T r = x OPER y;                                                      \
        if (r == r) return r;                                                \
        if (x != x) return Q(x);                                             \
        if (y != y) return Q(y);                                             \
        return D();                                                          \
    }
X86_OP(addf, float, +, qnan_f, dnan_f)
X86_OP(subf, float, -, qnan_f, dnan_f)
X86_OP(mulf, float, *, qnan_f, dnan_f)
X86_OP(addd, double, +, qnan_d, dnan_d)
X86_OP(subd, double, -, qnan_d, dnan_d)
X86_OP(muld, double, *, qnan_d, dnan_d)

static int do_sum(int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T, UT) case K: IWRAP_ADD(T, UT); return 0;
    INT_KINDS(X)
#undef X
    case ORK_F32: LOOP(float, b[i] = addf(b[i], a[i])); return 0;
    case ORK_F64: LOOP(double, b[i] = addd(b[i], a[i])); return 0;
    /* complex<T>::operator+= op.cpp:287-292 */
    case ORK_C32: LOOP(cplx_f, b[i].re = addf(b[i].re, a[i].re); b[i].im = addf(b[i].im, a[i].im)); return 0;
    case ORK_C64: LOOP(cplx_d, b[i].re = addd(b[i].re, a[i].re); b[i].im = addd(b[i].im, a[i].im)); return 0;
    default: return MPI_ERR_OP;
    }
}

/* complex<T>::operator*= op.cpp:294-303:
 *   r = (re * rhs.re) - (im * rhs.im);  i = (re * rhs.im) + (rhs.re * im); */
#define CMUL(T, ADD, SUB, MUL)                                               \
    LOOP(T, {                                                                \
        __typeof__(b[i].re) r = SUB(MUL(b[i].re, a[i].re), MUL(b[i].im, a[i].im)); \
        __typeof__(b[i].re) m = ADD(MUL(b[i].re, a[i].im), MUL(a[i].re, b[i].im)); \
        b[i].re = r; b[i].im = m; })

static int do_prod(int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T, UT) case K: IWRAP_MUL(T, UT); return 0;
    INT_KINDS(X)
#undef X
    case ORK_F32: LOOP(float, b[i] = mulf(b[i], a[i])); return 0;
    case ORK_F64: LOOP(double, b[i] = muld(b[i], a[i])); return 0;
    case ORK_C32: CMUL(cplx_f, addf, subf, mulf); return 0;
    case ORK_C64: CMUL(cplx_d, addd, subd, muld); return 0;
    default: return MPI_ERR_OP;
    }
}

/* logical ops: C truthiness (x != 0; NaN is true, -0.0 false), result T(0/1) */
#define LOGICAL_KINDS(X)                                                     \
    X(ORK_I8, int8_t) X(ORK_U8, uint8_t) X(ORK_I16, int16_t)                 \
    X(ORK_U16, uint16_t) X(ORK_I32, int32_t) X(ORK_U32, uint32_t)            \
    X(ORK_I64, int64_t) X(ORK_U64, uint64_t) X(ORK_F32, float)               \
    X(ORK_F64, double) X(ORK_BOOL, uint8_t)

static int do_logical(MPI_Op op, int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T)                                                              \
    case K:                                                                  \
        if (op == MPI_LAND) LOOP(T, b[i] = (T)((b[i] != 0) && (a[i] != 0)));  \
        else if (op == MPI_LOR) LOOP(T, b[i] = (T)((b[i] != 0) || (a[i] != 0))); \
        else LOOP(T, b[i] = (T)(((b[i] != 0) && !(a[i] != 0)) ||              \
                                (!(b[i] != 0) && (a[i] != 0))));              \
        return 0;
    LOGICAL_KINDS(X)
#undef X
    default: return MPI_ERR_OP;
    }
}

static int do_bitwise(MPI_Op op, int k, const void* in, void* inout, int64_t count)
{
    switch (k) {
#define X(K, T, UT)                                                          \
    case K:                                                                  \
        if (op == MPI_BAND) LOOP(T, b[i] &= a[i]);                           \
        else if (op == MPI_BOR) LOOP(T, b[i] |= a[i]);                       \
        else LOOP(T, b[i] ^= a[i]);                                          \
        return 0;
    INT_KINDS(X)
#undef X
    default: return MPI_ERR_OP;
    }
}

/* loctype<V,L>::MaxLoc / MinLoc (op.cpp:315-339): equal values keep the
 * smaller location (min() macro -> `in`'s on ties, identical anyway); otherwise
 * `*this = rhs` copies the whole struct, padding bytes included. */
#define LOCLOOP(T, CMP)                                                      \
    LOOP(T, {                                                                \
        if (b[i].v == a[i].v) {                                              \
            b[i].l = WMIN(b[i].l, a[i].l);                                   \
        } else if (CMP) {                                                    \
            memcpy(&b[i], &a[i], sizeof(T));                                 \
        } })

static int do_loc(MPI_Op op, int k, const void* in, void* inout, int64_t count)
{
    const int maxloc = (op == MPI_MAXLOC);
    switch (k) {
#define X(K, T)                                                              \
    case K:                                                                  \
        if (maxloc) LOCLOOP(T, b[i].v < a[i].v);                             \
        else LOCLOOP(T, b[i].v > a[i].v);                                    \
        return 0;
    X(ORK_LOC_II, loc_ii) X(ORK_LOC_FI, loc_fi) X(ORK_LOC_SI, loc_si)
    X(ORK_LOC_DI, loc_di) X(ORK_LOC_FF, loc_ff) X(ORK_LOC_DD, loc_dd)
#undef X
    default: return MPI_ERR_OP;
    }
}

int oracle_reduce_local(MPI_Op op, MPI_Datatype dt, const void* in, void* inout,
                        int64_t count)
{
    /* The reference switch only reaches a kernel for a legal pair; anything
     * else sets op_errno = MPI_ERR_OP (e.g. op.cpp:1791). */
    if (oracle_op_check(op, dt) != MPI_SUCCESS)
        return MPI_ERR_OP;
    if (count <= 0)
        return MPI_SUCCESS;
    int k = oracle_kind_of(dt);
    switch (op) {
    case MPI_MAX:  return do_max(k, in, inout, count);
    case MPI_MIN:  return do_min(k, in, inout, count);
    case MPI_SUM:  return do_sum(k, in, inout, count);
    case MPI_PROD: return do_prod(k, in, inout, count);
    case MPI_LAND: case MPI_LOR: case MPI_LXOR:
        return do_logical(op, k, in, inout, count);
    case MPI_BAND: case MPI_BOR: case MPI_BXOR:
        return do_bitwise(op, k, in, inout, count);
    case MPI_MAXLOC: case MPI_MINLOC:
        return do_loc(op, k, in, inout, count);
    default:
        return MPI_ERR_OP;
    }
}

/* ------------------------------------------------------------------------ */
/* multi-threaded CPU baseline: element range sharded over pthreads          */
/* ------------------------------------------------------------------------ */
typedef struct {
    MPI_Op op; MPI_Datatype dt; const char* in; char* inout; int64_t count;
    int rc;
} shard_t;

static void* shard_main(void* p)
{
    shard_t* s = (shard_t*)p;
    s->rc = oracle_reduce_local(s->op, s->dt, s->in, s->inout, s->count);
    return NULL;
}

int oracle_reduce_local_mt(MPI_Op op, MPI_Datatype dt, const void* in, void* inout,
                           int64_t count, int nthreads)
{
    if (nthreads <= 1 || count < nthreads)
        return oracle_reduce_local(op, dt, in, inout, count);
    int esz = oracle_kind_size(oracle_kind_of(dt));
    if (esz == 0)
        return MPI_ERR_OP;
    shard_t* sh = (shard_t*)calloc((size_t)nthreads, sizeof(shard_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    int64_t per = count / nthreads, rem = count % nthreads, off = 0;
    for (int t = 0; t < nthreads; ++t) {
        int64_t n = per + (t < rem ? 1 : 0);
        sh[t] = (shard_t){ op, dt, (const char*)in + off * esz, (char*)inout + off * esz, n, 0 };
        off += n;
        pthread_create(&th[t], NULL, shard_main, &sh[t]);
    }
    int rc = MPI_SUCCESS;
    for (int t = 0; t < nthreads; ++t) {
        pthread_join(th[t], NULL);
        if (sh[t].rc != MPI_SUCCESS) rc = sh[t].rc;
    }
    free(sh);
    free(th);
    return rc;
}
