// msx_types.cpp — predefined datatype table and (op, type) legality.
//
// Table rows follow src/include/mpi.h:284-368 (handle values) and the
// element type each row gets in op.cpp:343-536.  Legality follows
// op.cpp:739-1883.  See msx_types.h.
#include "msx_types.h"

namespace msx {

namespace {

const TypeInfo kTypes[] = {
    // C integers (CASE_MPI_C_INTS, op.cpp:343-398)
    {MPI_INT,                K_I32, G_CINT, 4, "MPI_INT"},
    {MPI_LONG,               K_I32, G_CINT, 4, "MPI_LONG"},           // LLP64
    {MPI_SHORT,              K_I16, G_CINT, 2, "MPI_SHORT"},
    {MPI_UNSIGNED_SHORT,     K_U16, G_CINT, 2, "MPI_UNSIGNED_SHORT"},
    {MPI_UNSIGNED,           K_U32, G_CINT, 4, "MPI_UNSIGNED"},
    {MPI_UNSIGNED_LONG,      K_U32, G_CINT, 4, "MPI_UNSIGNED_LONG"},  // LLP64
    {MPI_LONG_LONG,          K_I64, G_CINT, 8, "MPI_LONG_LONG"},
    {MPI_UNSIGNED_LONG_LONG, K_U64, G_CINT, 8, "MPI_UNSIGNED_LONG_LONG"},
    {MPI_SIGNED_CHAR,        K_I8,  G_CINT, 1, "MPI_SIGNED_CHAR"},
    {MPI_UNSIGNED_CHAR,      K_U8,  G_CINT, 1, "MPI_UNSIGNED_CHAR"},
    {MPI_INT8_T,             K_I8,  G_CINT, 1, "MPI_INT8_T"},
    {MPI_INT16_T,            K_I16, G_CINT, 2, "MPI_INT16_T"},
    {MPI_INT32_T,            K_I32, G_CINT, 4, "MPI_INT32_T"},
    {MPI_INT64_T,            K_I64, G_CINT, 8, "MPI_INT64_T"},
    {MPI_UINT8_T,            K_U8,  G_CINT, 1, "MPI_UINT8_T"},
    {MPI_UINT16_T,           K_U16, G_CINT, 2, "MPI_UINT16_T"},
    {MPI_UINT32_T,           K_U32, G_CINT, 4, "MPI_UINT32_T"},
    {MPI_UINT64_T,           K_U64, G_CINT, 8, "MPI_UINT64_T"},
    // Fortran integers (CASE_MPI_F_INTS, op.cpp:410-434)
    {MPI_INTEGER,            K_I32, G_FINT, 4, "MPI_INTEGER"},
    {MPI_AINT,               K_I64, G_FINT, 8, "MPI_AINT"},
    {MPI_OFFSET,             K_I64, G_FINT, 8, "MPI_OFFSET"},
    {MPI_INTEGER1,           K_I8,  G_FINT, 1, "MPI_INTEGER1"},
    {MPI_INTEGER2,           K_I16, G_FINT, 2, "MPI_INTEGER2"},
    {MPI_INTEGER4,           K_I32, G_FINT, 4, "MPI_INTEGER4"},
    {MPI_INTEGER8,           K_I64, G_FINT, 8, "MPI_INTEGER8"},
    // floating point (CASE_MPI_FLOATS, op.cpp:454-469); MSVC long double = double
    {MPI_FLOAT,              K_F32, G_FLOAT, 4, "MPI_FLOAT"},
    {MPI_REAL,               K_F32, G_FLOAT, 4, "MPI_REAL"},
    {MPI_REAL4,              K_F32, G_FLOAT, 4, "MPI_REAL4"},
    {MPI_DOUBLE,             K_F64, G_FLOAT, 8, "MPI_DOUBLE"},
    {MPI_DOUBLE_PRECISION,   K_F64, G_FLOAT, 8, "MPI_DOUBLE_PRECISION"},
    {MPI_REAL8,              K_F64, G_FLOAT, 8, "MPI_REAL8"},
    {MPI_LONG_DOUBLE,        K_F64, G_FLOAT, 8, "MPI_LONG_DOUBLE"},
    // complex (CASE_MPI_COMPLEXES, op.cpp:481-495)
    {MPI_COMPLEX8,           K_C32, G_COMPLEX, 8,  "MPI_COMPLEX8"},
    {MPI_COMPLEX,            K_C32, G_COMPLEX, 8,  "MPI_COMPLEX"},
    {MPI_C_COMPLEX,          K_C32, G_COMPLEX, 8,  "MPI_C_COMPLEX"},
    {MPI_C_FLOAT_COMPLEX,    K_C32, G_COMPLEX, 8,  "MPI_C_FLOAT_COMPLEX"},
    {MPI_COMPLEX16,          K_C64, G_COMPLEX, 16, "MPI_COMPLEX16"},
    {MPI_DOUBLE_COMPLEX,     K_C64, G_COMPLEX, 16, "MPI_DOUBLE_COMPLEX"},
    {MPI_C_DOUBLE_COMPLEX,   K_C64, G_COMPLEX, 16, "MPI_C_DOUBLE_COMPLEX"},
    {MPI_C_LONG_DOUBLE_COMPLEX, K_C64, G_COMPLEX, 16, "MPI_C_LONG_DOUBLE_COMPLEX"},
    // logicals (CASE_MPI_LOGICALS, op.cpp:498-504)
    {MPI_LOGICAL,            K_I32, G_LOGICAL, 4, "MPI_LOGICAL"},
    {MPI_C_BOOL,             K_BOOL, G_CBOOL, 1, "MPI_C_BOOL"},
    // byte (bitwise only, op.cpp:718)
    {MPI_BYTE,               K_U8,  G_BYTE, 1, "MPI_BYTE"},
    // printable chars (CASE_MPI_PRINTABLE_CHARS, op.cpp:507-511): signed char
    {MPI_CHAR,               K_I8,  G_PCHAR, 1, "MPI_CHAR"},
    {MPI_CHARACTER,          K_I8,  G_PCHAR, 1, "MPI_CHARACTER"},
    // value/location pairs (CASE_MPI_LOCTYPES, op.cpp:514-536)
    {MPI_2INT,               K_LOC_II, G_LOC, 8,  "MPI_2INT"},
    {MPI_2INTEGER,           K_LOC_II, G_LOC, 8,  "MPI_2INTEGER"},
    {MPI_LONG_INT,           K_LOC_II, G_LOC, 8,  "MPI_LONG_INT"},
    {MPI_FLOAT_INT,          K_LOC_FI, G_LOC, 8,  "MPI_FLOAT_INT"},
    {MPI_SHORT_INT,          K_LOC_SI, G_LOC, 8,  "MPI_SHORT_INT"},
    {MPI_DOUBLE_INT,         K_LOC_DI, G_LOC, 16, "MPI_DOUBLE_INT"},
    {MPI_LONG_DOUBLE_INT,    K_LOC_DI, G_LOC, 16, "MPI_LONG_DOUBLE_INT"},
    {MPI_2REAL,              K_LOC_FF, G_LOC, 8,  "MPI_2REAL"},
    {MPI_2DOUBLE_PRECISION,  K_LOC_DD, G_LOC, 16, "MPI_2DOUBLE_PRECISION"},
};

}  // namespace

const TypeInfo* type_info(MPI_Datatype dt)
{
    for (const TypeInfo& t : kTypes)
        if (t.handle == dt) return &t;
    return nullptr;
}

int type_size(MPI_Datatype dt)
{
    if (const TypeInfo* t = type_info(dt)) return t->size;
    switch (dt) {
    case MPI_WCHAR: return 2;
    case MPI_PACKED: return 1;
    case MPI_LB: case MPI_UB: return 0;
    case MPI_COUNT: return 8;
    case MPI_2COMPLEX: return 16;
    case MPI_2DOUBLE_COMPLEX: return 32;
    default: return -1;
    }
}

int kind_size(Kind k)
{
    switch (k) {
    case K_I8: case K_U8: case K_BOOL: return 1;
    case K_I16: case K_U16: return 2;
    case K_I32: case K_U32: case K_F32: return 4;
    case K_I64: case K_U64: case K_F64: case K_C32:
    case K_LOC_II: case K_LOC_FI: case K_LOC_SI: case K_LOC_FF: return 8;
    case K_C64: case K_LOC_DI: case K_LOC_DD: return 16;
    default: return 0;
    }
}

int op_legal_groups(int opidx)
{
    switch (opidx) {
    case O_MAX: case O_MIN:                 // op.cpp:1449-1521
        return G_CINT | G_FINT | G_FLOAT | G_PCHAR;
    case O_SUM: case O_PROD:                // op.cpp:1680-1883
        return G_CINT | G_FINT | G_FLOAT | G_COMPLEX | G_PCHAR;
    case O_LAND: case O_LOR: case O_LXOR:   // op.cpp:1026-1386
        return G_CINT | G_FINT | G_LOGICAL | G_CBOOL | G_FLOAT | G_PCHAR;
    case O_BAND: case O_BOR: case O_BXOR:   // op.cpp:739-1002
        return G_CINT | G_FINT | G_BYTE | G_LOGICAL | G_PCHAR;
    case O_MAXLOC: case O_MINLOC:           // op.cpp:1543-1571
        return G_LOC;
    default:
        return 0;
    }
}

int op_check_dtype(int opidx, MPI_Datatype dt)
{
    const TypeInfo* t = type_info(dt);
    if (t == nullptr) return MPI_ERR_OP;
    return (op_legal_groups(opidx) & t->group) ? MPI_SUCCESS : MPI_ERR_OP;
}

}  // namespace msx
