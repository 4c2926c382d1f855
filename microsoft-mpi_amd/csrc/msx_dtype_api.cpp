// msx_dtype_api.cpp — MPI datatype constructors, queries and MPI_Pack/Unpack.
//
// Argument checks keep the reference's order (the first failing check decides
// the error class a caller sees):
//   constructors / queries   api/mpi_datatype.cpp (cited per function)
//   MPI_Pack / Unpack / Pack_size  api/mpi_pack.cpp:41-500
//   MpiaDatatypeValidateHandle / Committed / NotPermanent  api/mpi_api.h:53-185
// The type objects and their flattened layouts live in msx_dtype.cpp; the
// byte movement of MPI_Pack / MPI_Unpack is the gfx950 kernel of msx_pack.hip
// (host operands are staged through HBM; there is no CPU packing path).
#include <limits.h>
#include <string.h>

#include <vector>

#include "../../include/mpi.h"
#include "msx_comm.h"
#include "msx_dtype.h"
#include "msx_runtime.h"
#include "msx_types.h"

using namespace msx;

#define MSX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kCombNamed = 1, kCombVector = 4, kCombHvectorInt = 5,
              kCombHvector = 6, kCombIndexed = 7, kCombHindexedInt = 8, kCombHindexed = 9,
              kCombIndexedBlock = 10, kCombStructInt = 11, kCombStruct = 12, kCombHindexedBlock = 19;

int fail(const char* fn, int code) { return api_err_return(fn, code); }

int arg_err(const char* what)
{
    set_error("%s", what);
    return MPI_ERR_ARG;
}

// MpiaDatatypeValidateHandle (mpi_api.h:53-72)
int v_handle(MPI_Datatype h, Dtype** out)
{
    if (h == MPI_DATATYPE_NULL) { set_error("null datatype"); return MPI_ERR_TYPE; }
    Dtype* t = dtype_lookup(h);
    if (!t) { set_error("invalid datatype 0x%x", h); return MPI_ERR_TYPE; }
    *out = t;
    return MPI_SUCCESS;
}

// MpiaDatatypeValidateNotPermanent (mpi_api.h:166-185)
int v_not_permanent(MPI_Datatype h)
{
    if (!dtype_is_derived(h)) { set_error("predefined datatype 0x%x", h); return MPI_ERR_TYPE; }
    return MPI_SUCCESS;
}

// MpiaDatatypeValidate (mpi_api.h:113-164), derived types included
int v_typed(const void* buf, int count, MPI_Datatype h, Dtype** out)
{
    *out = nullptr;
    if (count == 0) return MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); return MPI_ERR_COUNT; }
    int rc = v_handle(h, out);
    if (rc != MPI_SUCCESS) return rc;
    if (dtype_is_derived(h)) {
        if (!(*out)->committed) { set_error("datatype 0x%x is not committed", h); return MPI_ERR_TYPE; }
        if (buf == nullptr && (*out)->true_lb == 0 && (*out)->size > 0) { set_error("null buffer"); return MPI_ERR_BUFFER; }
    } else if (buf == nullptr) {
        set_error("null buffer");
        return MPI_ERR_BUFFER;
    }
    return MPI_SUCCESS;
}

}  // namespace

// ===========================================================================
// constructors
// ===========================================================================
// MPI_Type_contiguous (mpi_datatype.cpp:106-175)
MSX_EXPORT int MPI_Type_contiguous(int count, MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_contiguous");
    Dtype* o;
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (!newtype) rc = arg_err("null newtype");
    else rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS) rc = dtype_contiguous(count, oldtype, newtype);
    return fail("MPI_Type_contiguous", rc);
}

// MPI_Type_vector (mpi_datatype.cpp:3181-3260)
MSX_EXPORT int MPI_Type_vector(int count, int blocklength, int stride, MPI_Datatype oldtype,
                               MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_vector");
    Dtype* o;
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (blocklength < 0) rc = arg_err("negative blocklength");
    else rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_vector(count, blocklength, stride, false, oldtype, newtype, kCombVector);
    return fail("MPI_Type_vector", rc);
}

static int hvector_impl(const char* fn, int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                        MPI_Datatype* newtype, int combiner)
{
    api_require_init(fn);
    Dtype* o;
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (blocklength < 0) rc = arg_err("negative blocklength");
    else rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_vector(count, blocklength, stride, true, oldtype, newtype, combiner);
    return fail(fn, rc);
}

// MPI_Type_create_hvector; MPI_Type_hvector is its MPI-1 name
MSX_EXPORT int MPI_Type_create_hvector(int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                                       MPI_Datatype* newtype)
{
    return hvector_impl("MPI_Type_create_hvector", count, blocklength, stride, oldtype, newtype, kCombHvector);
}
MSX_EXPORT int MPI_Type_hvector(int count, int blocklength, MPI_Aint stride, MPI_Datatype oldtype,
                                MPI_Datatype* newtype)
{
    return hvector_impl("MPI_Type_hvector", count, blocklength, stride, oldtype, newtype, kCombHvectorInt);
}

static int indexed_checks(int count, const int* blens, const void* disps, MPI_Datatype oldtype)
{
    if (count < 0) { set_error("negative count %d", count); return MPI_ERR_COUNT; }
    if (count > 0 && !blens) return arg_err("null array_of_blocklengths");
    if (count > 0 && !disps) return arg_err("null array_of_displacements");
    Dtype* o;
    int rc = v_handle(oldtype, &o);
    if (rc != MPI_SUCCESS) return rc;
    for (int i = 0; i < count; ++i)
        if (blens[i] < 0) return arg_err("negative blocklength");
    return MPI_SUCCESS;
}

// MPI_Type_indexed (mpi_datatype.cpp: count, blocklens, indices, oldtype, blocklen >= 0, newtype)
MSX_EXPORT int MPI_Type_indexed(int count, const int array_of_blocklengths[], const int array_of_displacements[],
                                MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_indexed");
    int rc = indexed_checks(count, array_of_blocklengths, array_of_displacements, oldtype);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS)
        rc = dtype_indexed(count, array_of_blocklengths, array_of_displacements, false, oldtype, newtype,
                           kCombIndexed);
    return fail("MPI_Type_indexed", rc);
}

static int hindexed_impl(const char* fn, int count, const int* blens, const MPI_Aint* disps, MPI_Datatype oldtype,
                         MPI_Datatype* newtype, int combiner)
{
    api_require_init(fn);
    int rc = indexed_checks(count, blens, disps, oldtype);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_indexed(count, blens, disps, true, oldtype, newtype, combiner);
    return fail(fn, rc);
}

MSX_EXPORT int MPI_Type_create_hindexed(int count, const int array_of_blocklengths[],
                                        const MPI_Aint array_of_displacements[], MPI_Datatype oldtype,
                                        MPI_Datatype* newtype)
{
    return hindexed_impl("MPI_Type_create_hindexed", count, array_of_blocklengths, array_of_displacements, oldtype,
                         newtype, kCombHindexed);
}
MSX_EXPORT int MPI_Type_hindexed(int count, const int array_of_blocklengths[], const MPI_Aint array_of_displacements[],
                                 MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    return hindexed_impl("MPI_Type_hindexed", count, array_of_blocklengths, array_of_displacements, oldtype,
                         newtype, kCombHindexedInt);
}

// MPI_Type_create_indexed_block: count, blocklength, displacements, oldtype
MSX_EXPORT int MPI_Type_create_indexed_block(int count, int blocklength, const int array_of_displacements[],
                                             MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_create_indexed_block");
    Dtype* o;
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (blocklength < 0) rc = arg_err("negative blocklength");
    else if (count > 0 && !array_of_displacements) rc = arg_err("null array_of_displacements");
    else rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS)
        rc = dtype_indexed_block(count, blocklength, array_of_displacements, false, oldtype, newtype,
                                 kCombIndexedBlock);
    return fail("MPI_Type_create_indexed_block", rc);
}

MSX_EXPORT int MPI_Type_create_hindexed_block(int count, int blocklength, const MPI_Aint array_of_displacements[],
                                              MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_create_hindexed_block");
    Dtype* o;
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (blocklength < 0) rc = arg_err("negative blocklength");
    else if (count > 0 && !array_of_displacements) rc = arg_err("null array_of_displacements");
    else rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS)
        rc = dtype_indexed_block(count, blocklength, array_of_displacements, true, oldtype, newtype,
                                 kCombHindexedBlock);
    return fail("MPI_Type_create_hindexed_block", rc);
}

static int struct_impl(const char* fn, int count, const int* blens, const MPI_Aint* disps, const MPI_Datatype* types,
                       MPI_Datatype* newtype, int combiner)
{
    api_require_init(fn);
    int rc = MPI_SUCCESS;
    if (count < 0) { set_error("negative count %d", count); rc = MPI_ERR_COUNT; }
    else if (count > 0 && !blens) rc = arg_err("null array_of_blocklengths");
    else if (count > 0 && !disps) rc = arg_err("null array_of_displacements");
    else if (count > 0 && !types) rc = arg_err("null array_of_types");
    for (int i = 0; rc == MPI_SUCCESS && i < count; ++i) {
        if (blens[i] < 0) { rc = arg_err("negative blocklength"); break; }
        Dtype* o;
        rc = v_handle(types[i], &o);
    }
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_struct(count, blens, disps, types, newtype, combiner);
    return fail(fn, rc);
}

MSX_EXPORT int MPI_Type_create_struct(int count, const int array_of_blocklengths[],
                                      const MPI_Aint array_of_displacements[], const MPI_Datatype array_of_types[],
                                      MPI_Datatype* newtype)
{
    return struct_impl("MPI_Type_create_struct", count, array_of_blocklengths, array_of_displacements,
                       array_of_types, newtype, kCombStruct);
}
MSX_EXPORT int MPI_Type_struct(int count, const int array_of_blocklengths[], const MPI_Aint array_of_displacements[],
                               const MPI_Datatype array_of_types[], MPI_Datatype* newtype)
{
    return struct_impl("MPI_Type_struct", count, array_of_blocklengths, array_of_displacements, array_of_types,
                       newtype, kCombStructInt);
}

// MPI_Type_create_subarray (mpi_datatype.cpp:1390-1530)
MSX_EXPORT int MPI_Type_create_subarray(int ndims, const int array_of_sizes[], const int array_of_subsizes[],
                                        const int array_of_starts[], int order, MPI_Datatype oldtype,
                                        MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_create_subarray");
    int rc = MPI_SUCCESS;
    if (ndims <= 0) rc = arg_err("non-positive ndims");
    else if (!array_of_sizes) rc = arg_err("null array_of_sizes");
    else if (!array_of_subsizes) rc = arg_err("null array_of_subsizes");
    else if (!array_of_starts) rc = arg_err("null array_of_starts");
    for (int i = 0; rc == MPI_SUCCESS && i < ndims; ++i) {
        if (array_of_sizes[i] < 0) rc = arg_err("negative size");
        else if (array_of_subsizes[i] < 0) rc = arg_err("negative subsize");
        else if (array_of_starts[i] < 0) rc = arg_err("negative start");
        else if (array_of_subsizes[i] > array_of_sizes[i]) rc = arg_err("subsize larger than size");
        else if (array_of_starts[i] > array_of_sizes[i] - array_of_subsizes[i]) rc = arg_err("start out of range");
    }
    if (rc == MPI_SUCCESS && order != MPI_ORDER_C && order != MPI_ORDER_FORTRAN) rc = arg_err("invalid order");
    Dtype* o;
    if (rc == MPI_SUCCESS) rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS)
        rc = dtype_subarray(ndims, array_of_sizes, array_of_subsizes, array_of_starts, order, oldtype, newtype);
    return fail("MPI_Type_create_subarray", rc);
}

// MPI_Type_create_darray (mpi_datatype.cpp:218-600): the checks in the
// reference's order, then MPIR_Type_block / MPIR_Type_cyclic per dimension.
MSX_EXPORT int MPI_Type_create_darray(int size, int rank, int ndims, const int array_of_gsizes[],
                                      const int array_of_distribs[], const int array_of_dargs[],
                                      const int array_of_psizes[], int order, MPI_Datatype oldtype,
                                      MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_create_darray");
    Dtype* o;
    int rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && rank < 0) rc = arg_err("negative rank");
    if (rc == MPI_SUCCESS && size < 0) rc = arg_err("negative size");
    if (rc == MPI_SUCCESS && ndims < 0) rc = arg_err("negative ndims");
    if (rc == MPI_SUCCESS && !array_of_gsizes) rc = arg_err("null array_of_gsizes");
    if (rc == MPI_SUCCESS && !array_of_distribs) rc = arg_err("null array_of_distribs");
    if (rc == MPI_SUCCESS && !array_of_dargs) rc = arg_err("null array_of_dargs");
    if (rc == MPI_SUCCESS && !array_of_psizes) rc = arg_err("null array_of_psizes");
    if (rc == MPI_SUCCESS && order != MPI_ORDER_C && order != MPI_ORDER_FORTRAN) rc = arg_err("invalid order");
    for (int i = 0; rc == MPI_SUCCESS && i < ndims; ++i) {
        const int dist = array_of_distribs[i], darg = array_of_dargs[i];
        if (array_of_gsizes[i] < 0) rc = arg_err("negative gsize");
        else if (array_of_psizes[i] < 0) rc = arg_err("negative psize");
        else if (dist != MPI_DISTRIBUTE_NONE && dist != MPI_DISTRIBUTE_BLOCK && dist != MPI_DISTRIBUTE_CYCLIC)
            rc = arg_err("unknown distribution");
        else if (darg != MPI_DISTRIBUTE_DFLT_DARG && darg <= 0) rc = arg_err("invalid array_of_dargs");
        else if (dist == MPI_DISTRIBUTE_NONE && array_of_psizes[i] != 1)
            rc = arg_err("MPI_DISTRIBUTE_NONE needs a process-grid size of 1");
    }
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS)
        rc = dtype_darray(size, rank, ndims, array_of_gsizes, array_of_distribs, array_of_dargs, array_of_psizes,
                          order, oldtype, newtype);
    return fail("MPI_Type_create_darray", rc);
}

// MPI_Type_create_resized (mpi_datatype.cpp)
MSX_EXPORT int MPI_Type_create_resized(MPI_Datatype oldtype, MPI_Aint lb, MPI_Aint extent, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_create_resized");
    Dtype* o;
    int rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_resized(oldtype, lb, extent, newtype);
    return fail("MPI_Type_create_resized", rc);
}

// MPI_Type_dup
MSX_EXPORT int MPI_Type_dup(MPI_Datatype oldtype, MPI_Datatype* newtype)
{
    api_require_init("MPI_Type_dup");
    Dtype* o;
    int rc = v_handle(oldtype, &o);
    if (rc == MPI_SUCCESS && !newtype) rc = arg_err("null newtype");
    if (rc == MPI_SUCCESS) rc = dtype_dup(oldtype, newtype);
    return fail("MPI_Type_dup", rc);
}

// MPI_Type_commit: committing a predefined type is a no-op (the reference
// skips MPID_Type_commit when MpiaDatatypeValidateNotPermanent fails)
MSX_EXPORT int MPI_Type_commit(MPI_Datatype* datatype)
{
    api_require_init("MPI_Type_commit");
    if (!datatype) return fail("MPI_Type_commit", arg_err("null datatype"));
    Dtype* t;
    int rc = v_handle(*datatype, &t);
    if (rc == MPI_SUCCESS && dtype_is_derived(*datatype)) rc = dtype_commit(*datatype);
    return fail("MPI_Type_commit", rc);
}

MSX_EXPORT int MPI_Type_free(MPI_Datatype* datatype)
{
    api_require_init("MPI_Type_free");
    if (!datatype) return fail("MPI_Type_free", arg_err("null datatype"));
    Dtype* t;
    int rc = v_handle(*datatype, &t);
    if (rc == MPI_SUCCESS) rc = v_not_permanent(*datatype);
    if (rc == MPI_SUCCESS) rc = dtype_free(datatype);
    return fail("MPI_Type_free", rc);
}

// ===========================================================================
// queries
// ===========================================================================
MSX_EXPORT int MPI_Type_size(MPI_Datatype datatype, int* size)
{
    api_require_init("MPI_Type_size");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !size) rc = arg_err("null size");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_size", rc);
    *size = t->size > INT_MAX ? MPI_UNDEFINED : (int)t->size;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_size_x(MPI_Datatype datatype, MPI_Count* size)
{
    api_require_init("MPI_Type_size_x");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !size) rc = arg_err("null size");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_size_x", rc);
    *size = t->size;
    return MPI_SUCCESS;
}

// lb / extent of a predefined type are 0 / its size (pair types: struct extent)
static void lb_extent(const Dtype* t, MPI_Aint* lb, MPI_Aint* extent)
{
    *lb = t->lb;
    *extent = t->extent;
}

MSX_EXPORT int MPI_Type_get_extent(MPI_Datatype datatype, MPI_Aint* lb, MPI_Aint* extent)
{
    api_require_init("MPI_Type_get_extent");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !lb) rc = arg_err("null lb");
    if (rc == MPI_SUCCESS && !extent) rc = arg_err("null extent");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_extent", rc);
    lb_extent(t, lb, extent);
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_get_extent_x(MPI_Datatype datatype, MPI_Count* lb, MPI_Count* extent)
{
    api_require_init("MPI_Type_get_extent_x");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !lb) rc = arg_err("null lb");
    if (rc == MPI_SUCCESS && !extent) rc = arg_err("null extent");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_extent_x", rc);
    lb_extent(t, lb, extent);
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_get_true_extent(MPI_Datatype datatype, MPI_Aint* true_lb, MPI_Aint* true_extent)
{
    api_require_init("MPI_Type_get_true_extent");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !true_lb) rc = arg_err("null true_lb");
    if (rc == MPI_SUCCESS && !true_extent) rc = arg_err("null true_extent");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_true_extent", rc);
    *true_lb = t->true_lb;
    *true_extent = t->true_ub - t->true_lb;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_get_true_extent_x(MPI_Datatype datatype, MPI_Count* true_lb, MPI_Count* true_extent)
{
    api_require_init("MPI_Type_get_true_extent_x");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !true_lb) rc = arg_err("null true_lb");
    if (rc == MPI_SUCCESS && !true_extent) rc = arg_err("null true_extent");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_true_extent_x", rc);
    *true_lb = t->true_lb;
    *true_extent = t->true_ub - t->true_lb;
    return MPI_SUCCESS;
}

// MPI-1 forms (deprecated in the reference header, still exported)
MSX_EXPORT int MPI_Type_extent(MPI_Datatype datatype, MPI_Aint* extent)
{
    api_require_init("MPI_Type_extent");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !extent) rc = arg_err("null extent");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_extent", rc);
    *extent = t->extent;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_lb(MPI_Datatype datatype, MPI_Aint* displacement)
{
    api_require_init("MPI_Type_lb");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !displacement) rc = arg_err("null displacement");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_lb", rc);
    *displacement = t->lb;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_ub(MPI_Datatype datatype, MPI_Aint* displacement)
{
    api_require_init("MPI_Type_ub");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !displacement) rc = arg_err("null displacement");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_ub", rc);
    *displacement = t->ub;
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_get_envelope(MPI_Datatype datatype, int* num_integers, int* num_addresses,
                                     int* num_datatypes, int* combiner)
{
    api_require_init("MPI_Type_get_envelope");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && !num_integers) rc = arg_err("null num_integers");
    if (rc == MPI_SUCCESS && !num_addresses) rc = arg_err("null num_addresses");
    if (rc == MPI_SUCCESS && !num_datatypes) rc = arg_err("null num_datatypes");
    if (rc == MPI_SUCCESS && !combiner) rc = arg_err("null combiner");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_envelope", rc);
    if (!dtype_is_derived(datatype)) {
        *combiner = kCombNamed;
        *num_integers = *num_addresses = *num_datatypes = 0;
        return MPI_SUCCESS;
    }
    *combiner = t->combiner;
    *num_integers = (int)t->ints.size();
    *num_addresses = (int)t->aints.size();
    *num_datatypes = (int)t->types.size();
    return MPI_SUCCESS;
}

MSX_EXPORT int MPI_Type_get_contents(MPI_Datatype datatype, int max_integers, int max_addresses, int max_datatypes,
                                     int array_of_integers[], MPI_Aint array_of_addresses[],
                                     MPI_Datatype array_of_datatypes[])
{
    api_require_init("MPI_Type_get_contents");
    Dtype* t;
    int rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS) rc = v_not_permanent(datatype);
    if (rc == MPI_SUCCESS && max_integers > 0 && !array_of_integers) rc = arg_err("null array_of_integers");
    if (rc == MPI_SUCCESS && max_addresses > 0 && !array_of_addresses) rc = arg_err("null array_of_addresses");
    if (rc == MPI_SUCCESS && max_datatypes > 0 && !array_of_datatypes) rc = arg_err("null array_of_datatypes");
    // MPID_Type_get_contents: the caller's arrays must hold the whole envelope
    if (rc == MPI_SUCCESS && (max_integers < (int)t->ints.size() || max_addresses < (int)t->aints.size() ||
                              max_datatypes < (int)t->types.size()))
        rc = arg_err("contents arrays smaller than the envelope");
    if (rc != MPI_SUCCESS) return fail("MPI_Type_get_contents", rc);
    std::copy(t->ints.begin(), t->ints.end(), array_of_integers);
    std::copy(t->aints.begin(), t->aints.end(), array_of_addresses);
    for (size_t i = 0; i < t->types.size(); ++i) {
        array_of_datatypes[i] = t->types[i];
        dtype_add_ref(t->types[i]);      // derived types handed out hold a reference
    }
    return MPI_SUCCESS;
}

// MPI_Get_address / MPI_Address: the address as an integer (MPI_BOTTOM = 0)
MSX_EXPORT int MPI_Get_address(const void* location, MPI_Aint* address)
{
    api_require_init("MPI_Get_address");
    if (!address) return fail("MPI_Get_address", arg_err("null address"));
    *address = (MPI_Aint)(uintptr_t)location;
    return MPI_SUCCESS;
}
MSX_EXPORT int MPI_Address(void* location, MPI_Aint* address)
{
    api_require_init("MPI_Address");
    if (!address) return fail("MPI_Address", arg_err("null address"));
    *address = (MPI_Aint)(uintptr_t)location;
    return MPI_SUCCESS;
}

// ===========================================================================
// MPI_Pack / MPI_Unpack / MPI_Pack_size (api/mpi_pack.cpp)
// ===========================================================================
MSX_EXPORT int MPI_Pack(const void* inbuf, int incount, MPI_Datatype datatype, void* outbuf, int outsize,
                        int* position, MPI_Comm comm)
{
    api_require_init("MPI_Pack");
    ApiRange range("MPI_Pack");
    int rc = api_comm_valid(comm);
    Dtype* t = nullptr;
    if (rc == MPI_SUCCESS) rc = v_typed(inbuf, incount, datatype, &t);     // inbuf may be MPI_BOTTOM
    if (rc == MPI_SUCCESS && outsize < 0) rc = arg_err("negative outsize");
    if (rc == MPI_SUCCESS && incount > 0 && !outbuf) rc = arg_err("null outbuf");
    if (rc == MPI_SUCCESS && !position) rc = arg_err("null position");
    if (rc == MPI_SUCCESS && *position < 0) rc = arg_err("negative position");
    if (rc == MPI_SUCCESS && incount > 0 && t->size * (int64_t)incount > (int64_t)outsize - *position) {
        set_error("pack of %lld bytes into %lld", (long long)(t->size * (int64_t)incount),
                  (long long)((int64_t)outsize - *position));
        rc = MPI_ERR_ARG;
    }
    if (rc == MPI_SUCCESS && incount > 0) {
        rc = dt_pack_any(t, incount, inbuf, static_cast<char*>(outbuf) + *position);
        if (rc == MPI_SUCCESS) *position += (int)(t->size * (int64_t)incount);
    }
    return fail("MPI_Pack", rc);
}

MSX_EXPORT int MPI_Unpack(const void* inbuf, int insize, int* position, void* outbuf, int outcount,
                          MPI_Datatype datatype, MPI_Comm comm)
{
    api_require_init("MPI_Unpack");
    ApiRange range("MPI_Unpack");
    int rc = api_comm_valid(comm);                                       // mpi_pack.cpp:570-591
    Dtype* t = nullptr;
    if (rc == MPI_SUCCESS) rc = v_typed(outbuf, outcount, datatype, &t);
    if (rc == MPI_SUCCESS && !position) rc = arg_err("null position");
    if (rc == MPI_SUCCESS && insize < 0) { set_error("negative insize %d", insize); rc = MPI_ERR_COUNT; }
    if (rc != MPI_SUCCESS || insize == 0) return fail("MPI_Unpack", rc);  // :599-602
    if (!inbuf) return fail("MPI_Unpack", arg_err("null inbuf"));
    if (outcount == 0) return MPI_SUCCESS;
    // The reference unpacks outcount instances whatever insize says (reading
    // past the buffer); here a short input is an error instead.
    const int64_t need = t->size * (int64_t)outcount;
    if (need > (int64_t)insize - *position) {
        set_error("unpack of %lld bytes from %lld", (long long)need, (long long)((int64_t)insize - *position));
        return fail("MPI_Unpack", MPI_ERR_TRUNCATE);
    }
    if (need + *position > INT_MAX) { set_error("position overflow"); return fail("MPI_Unpack", MPI_ERR_SIZE); }
    rc = dt_unpack_any(t, outcount, static_cast<const char*>(inbuf) + *position, outbuf);
    if (rc == MPI_SUCCESS) *position += (int)need;
    return fail("MPI_Unpack", rc);
}

MSX_EXPORT int MPI_Pack_size(int incount, MPI_Datatype datatype, MPI_Comm comm, int* size)
{
    api_require_init("MPI_Pack_size");
    int rc = api_comm_valid(comm);
    Dtype* t = nullptr;
    if (rc == MPI_SUCCESS) rc = v_handle(datatype, &t);
    if (rc == MPI_SUCCESS && dtype_is_derived(datatype) && !t->committed) {
        set_error("datatype 0x%x is not committed", datatype);
        rc = MPI_ERR_TYPE;
    }
    if (rc == MPI_SUCCESS && incount < 0) { set_error("negative count %d", incount); rc = MPI_ERR_COUNT; }
    if (rc == MPI_SUCCESS && !size) rc = arg_err("null size");
    if (rc != MPI_SUCCESS) return fail("MPI_Pack_size", rc);
    const int64_t packsize = (int64_t)incount * t->size;   // mpi_pack.cpp:499-500
    *size = packsize > INT_MAX ? MPI_UNDEFINED : (int)packsize;
    return MPI_SUCCESS;
}

// ===========================================================================
// device-side extension ABI (include/msx.h)
// ===========================================================================
static int dev_typed_check(int64_t count, MPI_Datatype dt, Dtype** t)
{
    if (count < 0) { set_error("negative count"); return MPI_ERR_COUNT; }
    int rc = v_handle(dt, t);
    if (rc == MPI_SUCCESS && dtype_is_derived(dt) && !(*t)->committed) {
        set_error("datatype 0x%x is not committed", dt);
        rc = MPI_ERR_TYPE;
    }
    if (rc == MPI_SUCCESS) rc = ensure_device();
    return rc;
}

MSX_EXPORT int msx_pack_dev(const void* typed, int64_t count, MPI_Datatype datatype, void* packed, void* stream)
{
    Dtype* t;
    int rc = dev_typed_check(count, datatype, &t);
    if (rc != MPI_SUCCESS || count == 0) return rc;
    return dt_pack_dev(t, count, typed, packed, static_cast<hipStream_t>(stream));
}

MSX_EXPORT int msx_unpack_dev(const void* packed, int64_t count, MPI_Datatype datatype, void* typed, void* stream)
{
    Dtype* t;
    int rc = dev_typed_check(count, datatype, &t);
    if (rc != MPI_SUCCESS || count == 0) return rc;
    return dt_unpack_dev(t, count, packed, typed, static_cast<hipStream_t>(stream));
}

// ---- PMPI_ profiling aliases --------------------------------------------------
#define MSX_ALIAS(name) extern "C" __attribute__((visibility("default"), alias(#name)))
MSX_ALIAS(MPI_Type_contiguous) int PMPI_Type_contiguous(int, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_vector) int PMPI_Type_vector(int, int, int, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_hvector) int PMPI_Type_create_hvector(int, int, MPI_Aint, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_hvector) int PMPI_Type_hvector(int, int, MPI_Aint, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_indexed) int PMPI_Type_indexed(int, const int[], const int[], MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_hindexed) int PMPI_Type_create_hindexed(int, const int[], const MPI_Aint[], MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_hindexed) int PMPI_Type_hindexed(int, const int[], const MPI_Aint[], MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_indexed_block) int PMPI_Type_create_indexed_block(int, int, const int[], MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_hindexed_block) int PMPI_Type_create_hindexed_block(int, int, const MPI_Aint[], MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_struct) int PMPI_Type_create_struct(int, const int[], const MPI_Aint[], const MPI_Datatype[], MPI_Datatype*);
MSX_ALIAS(MPI_Type_struct) int PMPI_Type_struct(int, const int[], const MPI_Aint[], const MPI_Datatype[], MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_subarray) int PMPI_Type_create_subarray(int, const int[], const int[], const int[], int, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_darray) int PMPI_Type_create_darray(int, int, int, const int[], const int[], const int[], const int[], int, MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_create_resized) int PMPI_Type_create_resized(MPI_Datatype, MPI_Aint, MPI_Aint, MPI_Datatype*);
MSX_ALIAS(MPI_Type_dup) int PMPI_Type_dup(MPI_Datatype, MPI_Datatype*);
MSX_ALIAS(MPI_Type_commit) int PMPI_Type_commit(MPI_Datatype*);
MSX_ALIAS(MPI_Type_free) int PMPI_Type_free(MPI_Datatype*);
MSX_ALIAS(MPI_Type_size) int PMPI_Type_size(MPI_Datatype, int*);
MSX_ALIAS(MPI_Type_size_x) int PMPI_Type_size_x(MPI_Datatype, MPI_Count*);
MSX_ALIAS(MPI_Type_get_extent) int PMPI_Type_get_extent(MPI_Datatype, MPI_Aint*, MPI_Aint*);
MSX_ALIAS(MPI_Type_get_extent_x) int PMPI_Type_get_extent_x(MPI_Datatype, MPI_Count*, MPI_Count*);
MSX_ALIAS(MPI_Type_get_true_extent) int PMPI_Type_get_true_extent(MPI_Datatype, MPI_Aint*, MPI_Aint*);
MSX_ALIAS(MPI_Type_get_true_extent_x) int PMPI_Type_get_true_extent_x(MPI_Datatype, MPI_Count*, MPI_Count*);
MSX_ALIAS(MPI_Type_extent) int PMPI_Type_extent(MPI_Datatype, MPI_Aint*);
MSX_ALIAS(MPI_Type_lb) int PMPI_Type_lb(MPI_Datatype, MPI_Aint*);
MSX_ALIAS(MPI_Type_ub) int PMPI_Type_ub(MPI_Datatype, MPI_Aint*);
MSX_ALIAS(MPI_Type_get_envelope) int PMPI_Type_get_envelope(MPI_Datatype, int*, int*, int*, int*);
MSX_ALIAS(MPI_Type_get_contents) int PMPI_Type_get_contents(MPI_Datatype, int, int, int, int[], MPI_Aint[], MPI_Datatype[]);
MSX_ALIAS(MPI_Get_address) int PMPI_Get_address(const void*, MPI_Aint*);
MSX_ALIAS(MPI_Address) int PMPI_Address(void*, MPI_Aint*);
MSX_ALIAS(MPI_Pack) int PMPI_Pack(const void*, int, MPI_Datatype, void*, int, int*, MPI_Comm);
MSX_ALIAS(MPI_Unpack) int PMPI_Unpack(const void*, int, int*, void*, int, MPI_Datatype, MPI_Comm);
MSX_ALIAS(MPI_Pack_size) int PMPI_Pack_size(int, MPI_Datatype, MPI_Comm, int*);
