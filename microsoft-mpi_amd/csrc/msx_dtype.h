// msx_dtype.h — derived datatypes: type objects, the flattened layout the GPU
// walks, and the pack / unpack / accumulate entry points.
//
// What the reference does (src/mpi/msmpi/mpid/datatype.cpp, dataloop.cpp,
// segment.cpp): every constructor builds an MPID_Datatype (size, lb/ub with
// sticky markers, true_lb/true_ub, alignsize, eltype) and, at commit, a
// dataloop tree that MPID_Segment_pack/unpack interpret on the CPU, one
// contiguous piece at a time.
//
// What this does instead: the same type attributes, computed with the same
// formulas (MPID_DATATYPE_*_LB_UB, datatype.h:522-611; struct alignment
// padding, datatype.cpp:2142-2452), but the type map is flattened once into an
// ordered list of contiguous byte runs of ONE instance.  The gfx950 kernels
// (msx_pack.hip) map every packed granule straight to its address (a division
// for regular layouts, a binary search over run offsets otherwise), so a pack
// is one memory-bound launch with no interpreter state.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <mutex>
#include <vector>

#include "msx_types.h"

namespace msx {

struct DtRun {
    int64_t disp;    // byte offset of the run from the buffer address (may be < 0)
    int64_t len;     // bytes (> 0)
};

// Device view of one committed layout (plain data, passed by value to kernels).
struct DevLayout {
    int64_t size = 0;      // data bytes per instance (sum of run lengths)
    int64_t extent = 0;    // instance stride in bytes
    int64_t nruns = 0;
    // regular form: run k = [first + k*stride, +blen), k < nruns; with n1 > 0
    // (two levels) run k = [first + (k / n1)*stride2 + (k % n1)*stride, +blen)
    int regular = 0;
    int64_t first = 0, blen = 0, stride = 0;
    int64_t n1 = 0, stride2 = 0;
    // general form: disp[k], poff[k] = packed offset of run k (poff[nruns] = size)
    const int64_t* disp = nullptr;
    const int64_t* poff = nullptr;
    int align = 1;         // largest power of two <= 16 dividing every run disp / len, size, extent
};

struct Dtype {
    MPI_Datatype handle = MPI_DATATYPE_NULL;
    int refs = 1;
    bool committed = false;
    bool permanent = false;       // predefined (MpiaDatatypeValidateNotPermanent)
    int64_t size = 0, lb = 0, ub = 0, extent = 0, true_lb = 0, true_ub = 0;
    bool sticky_lb = false, sticky_ub = false;
    int64_t alignsize = 0;
    MPI_Datatype eltype = MPI_DATATYPE_NULL;   // basic element type, NULL when mixed
    int64_t el_size = 0;                       // -1 when mixed
    int64_t n_elements = 0;
    bool is_contig = false;
    std::vector<DtRun> runs;      // type map of one instance, in order, adjacent runs merged
    // Compact regular run list (a vector / hvector of a one-run type), kept
    // unmaterialised so huge strided types cost O(1) host memory: run k =
    // [rfirst + k*rstride, +rlen), k < rn; `runs` stays empty while rn > 0 and
    // is expanded only when another constructor needs the explicit list.
    // Two levels (rn2 > 1: a vector / hvector / contiguous of such a type with
    // one copy per block, e.g. the planes of a 3-D subarray): run (j, k) =
    // [rfirst + j*rstride2 + k*rstride, +rlen), j < rn2 outer, k < rn inner.
    int64_t rn = 0, rfirst = 0, rlen = 0, rstride = 0;
    int64_t rn2 = 1, rstride2 = 0;
    // MPI_Type_get_envelope / get_contents
    int combiner = 1;             // MPI_COMBINER_NAMED
    std::vector<int> ints;
    std::vector<MPI_Aint> aints;
    std::vector<MPI_Datatype> types;
    // device copy of the layout (built on first GPU use; guarded by the pool lock)
    DevLayout dev;
    bool dev_ready = false;
    void* dev_mem = nullptr;
};

// Lookup: predefined handles (including the pair types and MPI_LB/MPI_UB) and
// live derived types.  nullptr = not a datatype (MPI_ERR_TYPE).
Dtype* dtype_lookup(MPI_Datatype h);
bool dtype_is_derived(MPI_Datatype h);
// Data bytes of one instance (MPI_Type_size), -1 for an invalid handle.
int64_t dtype_size(MPI_Datatype h);
// Number of contiguous runs of one instance (compact or explicit form).
int64_t dtype_nruns(const Dtype* t);
// Visit the runs of one instance in type-map order (any form).
template <class F>
void dtype_for_each_run(const Dtype* t, F&& f)
{
    if (t->rn) {
        for (int64_t j = 0; j < t->rn2; ++j)
            for (int64_t k = 0; k < t->rn; ++k) f(t->rfirst + j * t->rstride2 + k * t->rstride, t->rlen);
    } else {
        for (const DtRun& r : t->runs) f(r.disp, r.len);
    }
}

// ---- constructors (argument checks are the caller's; return MPI error class)
// Each creates an uncommitted type and stores its handle in *out.
int dtype_contiguous(int count, MPI_Datatype old, MPI_Datatype* out);
int dtype_vector(int count, int blocklen, int64_t stride, bool stride_bytes, MPI_Datatype old,
                 MPI_Datatype* out, int combiner);
int dtype_indexed(int count, const int* blens, const void* disps, bool disp_bytes, MPI_Datatype old,
                  MPI_Datatype* out, int combiner);
int dtype_indexed_block(int count, int blen, const void* disps, bool disp_bytes, MPI_Datatype old,
                        MPI_Datatype* out, int combiner);
int dtype_struct(int count, const int* blens, const MPI_Aint* disps, const MPI_Datatype* types,
                 MPI_Datatype* out, int combiner);
int dtype_resized(MPI_Datatype old, int64_t lb, int64_t extent, MPI_Datatype* out);
int dtype_dup(MPI_Datatype old, MPI_Datatype* out);
int dtype_subarray(int ndims, const int* sizes, const int* subsizes, const int* starts, int order,
                   MPI_Datatype old, MPI_Datatype* out);
int dtype_darray(int size, int rank, int ndims, const int* gsizes, const int* distribs, const int* dargs,
                 const int* psizes, int order, MPI_Datatype old, MPI_Datatype* out);
int dtype_commit(MPI_Datatype h);
int dtype_free(MPI_Datatype* h);   // derived only (caller checked)
void dtype_add_ref(MPI_Datatype h);

// ---- data movement (stream-ordered on `s`; both buffers device-accessible) --
// packed[i*size + p] <- typed[i*extent + run(p)]
int dt_pack_dev(const Dtype* t, int64_t count, const void* typed, void* packed, hipStream_t s);
// typed[i*extent + run(p)] <- packed[i*size + p]
int dt_unpack_dev(const Dtype* t, int64_t count, const void* packed, void* typed, hipStream_t s);
// typed elem (op)= packed elem over the type map: the reference's
// do_accumulate_op on a derived target datatype (packethandling.cpp:2969-3004),
// op applied per element of t->eltype.  A type with no basic element type, or a
// pair outside the op's table, leaves `typed` unchanged (op_errno only).
int dt_acc_dev(int opidx, const Dtype* t, int64_t count, const void* packed, void* typed, hipStream_t s);

// Blocking forms that accept host (pageable or pinned) or device buffers.
int dt_pack_any(const Dtype* t, int64_t count, const void* typed, void* packed);
int dt_unpack_any(const Dtype* t, int64_t count, const void* packed, void* typed);
// MPIR_Localcopy (mpid/pt2pt.cpp:770-948): typed -> typed with matching data
// sizes (the smaller one is copied, MPI_ERR_TRUNCATE when the receive is smaller).
int dt_copy_any(const void* src, int64_t scount, MPI_Datatype sdt, void* dst, int64_t rcount,
                MPI_Datatype rdt);

// Serialized layout of a type (size, extent, eltype, nruns, runs...) and the
// standalone (handle-less) type rebuilt from it at a one-sided target.
void dtype_serialize(const Dtype* t, std::vector<int64_t>& out);
Dtype* dtype_from_blob(const int64_t* blob, int64_t avail);   // nullptr when malformed
void dtype_delete(Dtype* t);                                   // standalone types only

// Byte span touched by `count` instances: [lo, hi) relative to the buffer.
void dt_span(const Dtype* t, int64_t count, int64_t* lo, int64_t* hi);

// ---- entry-point helpers (msx_api.cpp) -------------------------------------
void api_require_init(const char* fn);              // MpiaIsInitializedOrExit
int api_err_return(const char* fn, int code);       // MPIR_Err_return_comm(NULL, ...)
int api_comm_valid(MPI_Comm comm);                   // MpiaCommValidateHandle

}  // namespace msx
