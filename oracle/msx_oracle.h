/*
 * msx_oracle.h — CPU restatement of MS-MPI's MPI_Op kernels (TEST INFRASTRUCTURE).
 *
 * ORACLE — test infrastructure only.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this library.  The product path
 * (libmsmpi_mi355x.so) never links or calls it.
 *
 * Parity pinning: the reference library cannot be built here (op.cpp pulls
 * precomp.h -> mpiimpl.h -> windows.h/winsock2.h/SAL/ETW, which this image
 * lacks and which must not be replaced by stand-ins), so oracle/_ref does not
 * exist.  The restatement is checked against the known-answer outputs the
 * survey recorded from op.cpp built with a probe shim (SURVEY.md §8(a) notes /
 * Appendix A, committed as tests/golden/survey_kat.json).  A shim build does
 * not count as a reference build in this task, so: PARITY UNPINNED (DESIGN.md
 * §2), with x86 silicon as an independent anchor for the float / NaN rules.
 */
#ifndef MSX_ORACLE_H
#define MSX_ORACLE_H

#include <stdint.h>
#include "../include/mpi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Element classes the reference's CASE_MPI_* macros map datatypes to
 * (op.cpp:343-536; LLP64 widths per mpi.h:284-368). */
enum oracle_kind {
    ORK_NONE = 0,
    ORK_I8, ORK_U8, ORK_I16, ORK_U16, ORK_I32, ORK_U32, ORK_I64, ORK_U64,
    ORK_F32, ORK_F64, ORK_BOOL, ORK_C32, ORK_C64,
    ORK_LOC_II, ORK_LOC_FI, ORK_LOC_SI, ORK_LOC_DI, ORK_LOC_FF, ORK_LOC_DD,
    ORK_COUNT
};

/* datatype handle -> element class (ORK_NONE if not reducible) */
int oracle_kind_of(MPI_Datatype dt);
/* bytes per element of a kind (sizeof the C struct, padding included): the
 * datatype's EXTENT */
int oracle_kind_size(int kind);
/* MPI_Type_size (data bytes; 12 for MPI_DOUBLE_INT, 6 for MPI_SHORT_INT,
 * datatype.cpp:1282-1293) */
int oracle_type_size(MPI_Datatype dt);
/* MPIR_Op_<op>_check_dtype (op.cpp:739-1883): MPI_SUCCESS or MPI_ERR_OP */
int oracle_op_check(MPI_Op op, MPI_Datatype dt);
/* MPIR_Op_<op>(in, inout, &len, &dt) (op.cpp:703-1795) with a 64-bit count.
 * Returns the value the reference leaves in op_errno: MPI_SUCCESS, or
 * MPI_ERR_OP for an unsupported (op, type) pair (inout untouched). */
int oracle_reduce_local(MPI_Op op, MPI_Datatype dt, const void* in, void* inout,
                        int64_t count);

/* CPU baseline helper: sharded over nthreads pthreads (1 = one MS-MPI rank). */
int oracle_reduce_local_mt(MPI_Op op, MPI_Datatype dt, const void* in, void* inout,
                           int64_t count, int nthreads);

/* Reference-order multi-rank schedules (restated from mpid/reduce.cpp), used as
 * the expected result of the collectives for p ranks.  sendbufs[r] is rank r's
 * contribution (count elements each); results are written per rank.
 * Returns MPI_SUCCESS / MPI_ERR_OP / MPI_ERR_ARG. */
int oracle_allreduce(MPI_Op op, MPI_Datatype dt, int p, int64_t count,
                     const void* const* sendbufs, void* const* recvbufs);
int oracle_reduce_scatter(MPI_Op op, MPI_Datatype dt, int p, const int* recvcounts,
                          const void* const* sendbufs, void* const* recvbufs);
int oracle_reduce(MPI_Op op, MPI_Datatype dt, int p, int root, int64_t count,
                  const void* const* sendbufs, void* recvbuf_root);
int oracle_scan(MPI_Op op, MPI_Datatype dt, int p, int64_t count, int exclusive,
                const void* const* sendbufs, void* const* recvbufs);
/* The non-blocking forms as the reference builds their NBC task lists (also
 * what MSMPI_FORCE_ASYNC_WORKFLOW runs for the blocking calls):
 *  - MPI_Iallreduce, IallreduceBuildTaskList (reduce.cpp:4699-4982): the
 *    blocking butterfly, but the Rabenseifner gate reads the EXTENT,
 *    (unsigned)(extent*count) > short_msg (:4717, :4791, :4881), where the
 *    blocking call reads MPI_Type_size (:3884);
 *  - MPI_Ireduce, IreduceBuildTaskList (:6676-6768): the same extent gate
 *    (:6740), and IreduceBuildScatterGatherTaskList (:6267-6670) runs the
 *    recursive halving over ranks RELATIVE TO THE ROOT (odd relative ranks
 *    fold into relativeRank-1, TrimmedToOriginalRankEven, peers at
 *    root + relative rank), where the blocking Rabenseifner uses absolute
 *    ranks (:174-300).  The binomial task list (:6005-6198) equals the
 *    blocking binomial tree.
 *  - MPI_Ireduce_scatter[_block] (:3176-3257) gate on MPI_Type_size like the
 *    blocking call and build the same trees, so oracle_reduce_scatter serves. */
int oracle_iallreduce(MPI_Op op, MPI_Datatype dt, int p, int64_t count,
                      const void* const* sendbufs, void* const* recvbufs);
int oracle_ireduce(MPI_Op op, MPI_Datatype dt, int p, int root, int64_t count,
                   const void* const* sendbufs, void* recvbuf_root);

/* CPU baseline of the collective configs (msx_oracle_threads.c): p threads as
 * the p ranks of one host running the reference's step loop for their own
 * rank.  which 0: Rabenseifner allreduce of `count` elements per rank;
 * which 1: recursive-halving reduce_scatter_block of `count` per rank.
 * p a power of two; dt MPI_FLOAT / MPI_DOUBLE / MPI_UINT64_T.  times[rep]
 * receives each call's seconds; the result is checked on a sample. */
int oracle_coll_threads(int which, MPI_Op op, MPI_Datatype dt, int p, int64_t count, int reps, double* times);

#ifdef __cplusplus
}
#endif
#endif
