/*
 * op_table_test.c — the builtin op table driven the way the reference's
 * internal callers drive MPIR_Op_table (src/mpi/msmpi/mpid/op.cpp:618-622):
 * fetch the MPI_User_function of an op handle, call it with
 * (in, inout, &len, &datatype) on DEVICE buffers, read op_errno.
 *
 * Plain C against include/mpi.h + include/msx.h, linked with
 * libmsmpi_mi355x.so; the expected values come from the oracle
 * (oracle/liboracle.so, test infrastructure) on host copies of the same
 * inputs.  Every legal (op, datatype) pair of the predefined types is
 * compared byte for byte; every illegal pair must leave inout untouched and
 * set op_errno to MPI_ERR_OP; *len <= 0 must do nothing.  Prints "OK <pairs>"
 * and exits 0 on success.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "mpi.h"
#include "msx.h"
#include "../../oracle/msx_oracle.h"

static const MPI_Op kOps[] = {MPI_MAX, MPI_MIN, MPI_SUM, MPI_PROD, MPI_LAND, MPI_BAND,
                              MPI_LOR, MPI_BOR, MPI_LXOR, MPI_BXOR, MPI_MINLOC, MPI_MAXLOC};
static MPI_User_function* const kEntries[] = {msx_op_max, msx_op_min, msx_op_sum, msx_op_prod,
                                              msx_op_land, msx_op_band, msx_op_lor, msx_op_bor,
                                              msx_op_lxor, msx_op_bxor, msx_op_minloc, msx_op_maxloc};

static const MPI_Datatype kTypes[] = {
    MPI_INT, MPI_LONG, MPI_SHORT, MPI_UNSIGNED_SHORT, MPI_UNSIGNED, MPI_UNSIGNED_LONG, MPI_LONG_LONG,
    MPI_UNSIGNED_LONG_LONG, MPI_SIGNED_CHAR, MPI_UNSIGNED_CHAR, MPI_INT8_T, MPI_INT16_T, MPI_INT32_T,
    MPI_INT64_T, MPI_UINT8_T, MPI_UINT16_T, MPI_UINT32_T, MPI_UINT64_T, MPI_INTEGER, MPI_AINT, MPI_OFFSET,
    MPI_INTEGER1, MPI_INTEGER2, MPI_INTEGER4, MPI_INTEGER8, MPI_FLOAT, MPI_REAL, MPI_REAL4, MPI_DOUBLE,
    MPI_DOUBLE_PRECISION, MPI_REAL8, MPI_LONG_DOUBLE, MPI_COMPLEX8, MPI_COMPLEX, MPI_C_COMPLEX,
    MPI_C_FLOAT_COMPLEX, MPI_COMPLEX16, MPI_DOUBLE_COMPLEX, MPI_C_DOUBLE_COMPLEX, MPI_C_LONG_DOUBLE_COMPLEX,
    MPI_LOGICAL, MPI_C_BOOL, MPI_BYTE, MPI_CHAR, MPI_CHARACTER, MPI_2INT, MPI_2INTEGER, MPI_LONG_INT,
    MPI_FLOAT_INT, MPI_SHORT_INT, MPI_DOUBLE_INT, MPI_LONG_DOUBLE_INT, MPI_2REAL, MPI_2DOUBLE_PRECISION,
    /* predefined, never reducible with builtin ops */
    MPI_WCHAR, MPI_PACKED, MPI_COUNT, MPI_2COMPLEX};

static uint64_t g_rng = 0x5EEDull;
static uint64_t next64(void)
{
    g_rng += 0x9E3779B97F4A7C15ull;   /* splitmix64 */
    uint64_t z = g_rng;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* edge-heavy values: ties, zeros of both signs, NaN, infinities, wrap */
static double fval(void)
{
    static const double e[] = {0.0, -0.0, NAN, INFINITY, -INFINITY, 1.0, -1.0, 2.5, 3.0, 3.0, -7.25, 1e-310};
    const uint64_t r = next64();
    if (r % 3 == 0) return e[(r >> 8) % (sizeof(e) / sizeof(e[0]))];
    return ((double)((int64_t)(r >> 11) % 2000001) - 1000000.0) / 997.0;
}

static void fill(MPI_Datatype dt, unsigned char* b, int n)
{
    const int k = oracle_kind_of(dt), esz = oracle_kind_size(k);
    for (int i = 0; i < n; ++i) {
        unsigned char* e = b + (size_t)i * esz;
        for (int j = 0; j < esz; ++j) e[j] = (unsigned char)next64();   /* padding random too */
        switch (k) {
        case ORK_I8: case ORK_U8: case ORK_I16: case ORK_U16: case ORK_I32: case ORK_U32:
        case ORK_I64: case ORK_U64:
            if (next64() % 4 == 0) memset(e, 0, (size_t)esz);              /* zeros for the logical ops */
            else if (next64() % 5 == 0) { memset(e, 0, (size_t)esz); e[0] = 7; }   /* ties */
            break;
        case ORK_BOOL: e[0] = (unsigned char)(next64() & 1); break;
        case ORK_F32: { float f = (float)fval(); memcpy(e, &f, 4); break; }
        case ORK_F64: { double d = fval(); memcpy(e, &d, 8); break; }
        case ORK_C32: { float f[2] = {(float)fval(), (float)fval()}; memcpy(e, f, 8); break; }
        case ORK_C64: { double d[2] = {fval(), fval()}; memcpy(e, d, 16); break; }
        case ORK_LOC_II: { int32_t v[2] = {(int32_t)(next64() % 7) - 3, (int32_t)(next64() % 100) - 50}; memcpy(e, v, 8); break; }
        case ORK_LOC_FI: { float v = (float)((int)(next64() % 7) - 3); int32_t l = (int32_t)(next64() % 100) - 50;
                           if (next64() % 20 == 0) { v = NAN; }
                           memcpy(e, &v, 4); memcpy(e + 4, &l, 4); break; }
        case ORK_LOC_SI: { int16_t v = (int16_t)((int)(next64() % 7) - 3); int32_t l = (int32_t)(next64() % 100) - 50;
                           memcpy(e, &v, 2); memcpy(e + 4, &l, 4); break; }
        case ORK_LOC_DI: { double v = (double)((int)(next64() % 7) - 3); int32_t l = (int32_t)(next64() % 100) - 50;
                           if (next64() % 20 == 0) { v = NAN; }
                           memcpy(e, &v, 8); memcpy(e + 8, &l, 4); break; }
        case ORK_LOC_FF: { float v[2] = {(float)((int)(next64() % 7) - 3), (float)((int)(next64() % 100) - 50)};
                           if (next64() % 20 == 0) { v[0] = NAN; }
                           memcpy(e, v, 8); break; }
        case ORK_LOC_DD: { double v[2] = {(double)((int)(next64() % 7) - 3), (double)((int)(next64() % 100) - 50)};
                           if (next64() % 20 == 0) { v[0] = NAN; }
                           memcpy(e, v, 16); break; }
        default: break;
        }
    }
}

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 3; } } while (0)

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    int fails = 0, pairs = 0, illegal = 0;
    const int n = 4099;                                  /* a ragged count: vector body + tail */
    const size_t cap = (size_t)n * 32;
    unsigned char *hin = malloc(cap), *hio = malloc(cap), *exp = malloc(cap), *got = malloc(cap);
    void *din = NULL, *dio = NULL;
    CHECK_HIP(hipMalloc(&din, cap));
    CHECK_HIP(hipMalloc(&dio, cap));

    /* the table: MPIR_Op_table[op % 16 - 1] */
    for (int o = 0; o < 12; ++o)
        if (msx_op_table(kOps[o]) != kEntries[o]) { fprintf(stderr, "table entry %d\n", o); ++fails; }
    if (msx_op_table(MPI_REPLACE) != msx_op_replace || msx_op_table(MPI_NO_OP) != msx_op_noop ||
        msx_op_table(MPI_OP_NULL) != NULL || msx_op_table((MPI_Op)0x5800000f) != NULL ||
        msx_op_table((MPI_Op)0x58000101) != NULL) {
        fprintf(stderr, "table lookup of non-reduction handles\n");
        ++fails;
    }

    for (int o = 0; o < 12; ++o) {
        for (size_t t = 0; t < sizeof(kTypes) / sizeof(kTypes[0]); ++t) {
            MPI_Datatype dt = kTypes[t];
            const int k = oracle_kind_of(dt);
            const int esz = k ? oracle_kind_size(k) : 8;
            const size_t bytes = (size_t)n * (size_t)esz;
            if (k) { fill(dt, hin, n); fill(dt, hio, n); }
            else { for (size_t i = 0; i < bytes; ++i) { hin[i] = (unsigned char)next64(); hio[i] = (unsigned char)next64(); } }
            memcpy(exp, hio, bytes);
            const int legal = oracle_op_check(kOps[o], dt) == MPI_SUCCESS;
            if (legal) oracle_reduce_local(kOps[o], dt, hin, exp, n);
            CHECK_HIP(hipMemcpy(din, hin, bytes, hipMemcpyHostToDevice));
            CHECK_HIP(hipMemcpy(dio, hio, bytes, hipMemcpyHostToDevice));
            msx_op_errno_reset();
            int len = n;
            MPI_Datatype d = dt;
            MPI_User_function* f = msx_op_table(kOps[o]);
            f(din, dio, &len, &d);
            const int err = msx_op_errno();
            CHECK_HIP(hipMemcpy(got, dio, bytes, hipMemcpyDeviceToHost));
            if (legal) {
                ++pairs;
                if (err != MPI_SUCCESS || memcmp(got, exp, bytes) != 0) {
                    fprintf(stderr, "op %d type 0x%x: errno %d, result %s\n", o, (unsigned)dt, err,
                            memcmp(got, exp, bytes) ? "differs" : "ok");
                    ++fails;
                }
            } else {
                ++illegal;
                if (err != MPI_ERR_OP || memcmp(got, hio, bytes) != 0) {
                    fprintf(stderr, "illegal op %d type 0x%x: errno %d (want %d), inout %s\n", o, (unsigned)dt, err,
                            MPI_ERR_OP, memcmp(got, hio, bytes) ? "changed" : "untouched");
                    ++fails;
                }
            }
        }
    }

    /* *len <= 0 does nothing (while (--len >= 0) runs no iteration) */
    {
        fill(MPI_INT, hin, n); fill(MPI_INT, hio, n);
        CHECK_HIP(hipMemcpy(din, hin, (size_t)n * 4, hipMemcpyHostToDevice));
        CHECK_HIP(hipMemcpy(dio, hio, (size_t)n * 4, hipMemcpyHostToDevice));
        int len = 0, neg = -5;
        MPI_Datatype d = MPI_INT;
        msx_op_errno_reset();
        msx_op_sum(din, dio, &len, &d);
        msx_op_sum(din, dio, &neg, &d);
        CHECK_HIP(hipMemcpy(got, dio, (size_t)n * 4, hipMemcpyDeviceToHost));
        if (msx_op_errno() != 0 || memcmp(got, hio, (size_t)n * 4) != 0) { fprintf(stderr, "len <= 0\n"); ++fails; }
    }
    /* op_errno is sticky until reset, as the reference's per-call-state field */
    {
        int len = 4;
        MPI_Datatype d = MPI_BYTE;
        msx_op_errno_reset();
        msx_op_sum(din, dio, &len, &d);          /* SUM on MPI_BYTE: MPI_ERR_OP */
        d = MPI_INT;
        msx_op_sum(din, dio, &len, &d);          /* a good call does not clear it */
        if (msx_op_errno() != MPI_ERR_OP) { fprintf(stderr, "op_errno not sticky\n"); ++fails; }
        msx_op_errno_reset();
        if (msx_op_errno() != 0) { fprintf(stderr, "op_errno reset\n"); ++fails; }
    }
    /* the binding's routing test: device pairs only */
    if (msx_operands_on_device(din, dio) != 1 || msx_operands_on_device(hin, dio) != 0 ||
        msx_operands_on_device(din, hio) != 0 || msx_operands_on_device(NULL, dio) != 0) {
        fprintf(stderr, "msx_operands_on_device\n");
        ++fails;
    }
    /* host operands: offloaded like MPI_Reduce_local; MPI_REPLACE copies */
    {
        fill(MPI_DOUBLE, hin, n); fill(MPI_DOUBLE, hio, n);
        memcpy(exp, hio, (size_t)n * 8);
        oracle_reduce_local(MPI_MAX, MPI_DOUBLE, hin, exp, n);
        int len = n;
        MPI_Datatype d = MPI_DOUBLE;
        msx_op_errno_reset();
        msx_op_table(MPI_MAX)(hin, hio, &len, &d);
        if (msx_op_errno() != 0 || memcmp(hio, exp, (size_t)n * 8) != 0) { fprintf(stderr, "host MAX\n"); ++fails; }
        msx_op_table(MPI_REPLACE)(hin, hio, &len, &d);
        if (memcmp(hio, hin, (size_t)n * 8) != 0) { fprintf(stderr, "host REPLACE\n"); ++fails; }
        memcpy(exp, hio, (size_t)n * 8);
        msx_op_table(MPI_NO_OP)(hin, hio, &len, &d);
        if (memcmp(hio, exp, (size_t)n * 8) != 0) { fprintf(stderr, "NO_OP\n"); ++fails; }
    }

    (void)hipFree(din);
    (void)hipFree(dio);
    free(hin); free(hio); free(exp); free(got);
    MPI_Finalize();
    if (fails) { fprintf(stderr, "%d failures\n", fails); return 1; }
    printf("OK %d legal pairs, %d illegal pairs\n", pairs, illegal);
    return 0;
}
