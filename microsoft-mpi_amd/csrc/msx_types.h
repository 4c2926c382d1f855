// msx_types.h — datatype/op tables for the MI355X reduction path.
//
// Product code (not the oracle).  Restates, for the device dispatch:
//   * the datatype -> element-class map of MS-MPI's CASE_MPI_* macros
//     (/root/reference/src/mpi/msmpi/mpid/op.cpp:343-536) with the LLP64 widths
//     of the reference header (src/include/mpi.h:284-368);
//   * the (op, datatype) legality tables MPIR_Op_<op>_check_dtype
//     (op.cpp:739-1883, USE_STRICT_MPI undefined) reached through
//     MPIR_Op_check_dtype_table[op % 16 - 1] (op.cpp:653-672).
#pragma once

#include <stdint.h>
#include "../../include/mpi.h"

namespace msx {

// Element classes.  Every legal (op, datatype) pair runs one device kernel
// instantiated on one of these.
enum Kind : int {
    K_NONE = 0,
    K_I8, K_U8, K_I16, K_U16, K_I32, K_U32, K_I64, K_U64,
    K_F32, K_F64, K_BOOL, K_C32, K_C64,
    K_LOC_II, K_LOC_FI, K_LOC_SI, K_LOC_DI, K_LOC_FF, K_LOC_DD,
    K_COUNT
};

// Builtin op index = HANDLE_BUILTIN_INDEX(op) (mpihandlemem.h:236), 1..14.
enum OpIdx : int {
    O_NULL = 0, O_MAX = 1, O_MIN, O_SUM, O_PROD, O_LAND, O_BAND, O_LOR, O_BOR,
    O_LXOR, O_BXOR, O_MINLOC, O_MAXLOC, O_REPLACE, O_NOOP, O_COUNT
};

// Handle layout (src/mpi/common/mpihandlemem.h:175-236):
//   bits 31..30 type (0 invalid, 1 builtin, 2 direct, 3 indirect)
//   bits 29..26 object kind (MPID_OP = 6, MPID_DATATYPE = 3)
constexpr int handle_type(int h) { return (int)(((unsigned)h & 0xc0000000u) >> 30); }
constexpr int handle_kind(int h) { return (int)(((unsigned)h & 0x3c000000u) >> 26); }
constexpr int HT_INVALID = 0, HT_BUILTIN = 1, HT_DIRECT = 2;
constexpr int OBJ_OP = 6;

// Legality groups of the check tables.
enum Group : int {
    G_CINT = 1, G_FINT = 2, G_FLOAT = 4, G_COMPLEX = 8, G_LOGICAL = 16,
    G_CBOOL = 32, G_BYTE = 64, G_PCHAR = 128, G_LOC = 256
};

struct TypeInfo {
    MPI_Datatype handle;
    Kind kind;
    int group;
    int size;          // bytes per element (struct size, padding included)
    const char* name;
};

// Returns nullptr for handles that are not predefined reducible types.
const TypeInfo* type_info(MPI_Datatype dt);
// Size in bytes of a predefined datatype (any predefined, including
// non-reducible ones such as MPI_WCHAR); -1 if unknown.
int type_size(MPI_Datatype dt);
int kind_size(Kind k);
// Groups each builtin op accepts (the *_check_dtype switch bodies).
int op_legal_groups(int opidx);
// MPIR_Op_check_dtype_table[op%16-1](dt): MPI_SUCCESS or MPI_ERR_OP.
int op_check_dtype(int opidx, MPI_Datatype dt);

}  // namespace msx
