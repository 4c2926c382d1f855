/*
 * msx.h — device-side C ABI of the MI355X MS-MPI reduction path.
 *
 * Plain C, no HIP/torch types: streams are passed as `void*` (a hipStream_t,
 * NULL = the HIP null stream, as with any HIP API).
 *
 * Each entry point names the reference interface it replaces:
 *
 *   msx_reduce_local_dev  <- MPID_Uop_call(op, in, inout, &len, &dt)
 *                            (src/mpi/msmpi/include/op.h:171-174) reaching
 *                            MPIR_Op_<op>(void*, void*, int*, MPI_Datatype*)
 *                            (src/mpi/msmpi/mpid/op.cpp:703-1795), with the
 *                            MPI_Reduce_local argument checks
 *                            (src/mpi/msmpi/api/mpi_reduce.cpp:304-385);
 *                            64-bit count, stream-ordered, device pointers.
 *   msx_op_check          <- MPIR_Op_check_dtype_table[op%16-1](dt)
 *                            (op.cpp:653-672, api/mpi_api.h:765)
 *   msx_pack_dev /        <- MPID_Segment_pack / MPID_Segment_unpack over a
 *   msx_unpack_dev           committed datatype (src/mpi/msmpi/mpid/segment.cpp,
 *                            called by MPI_Pack/MPI_Unpack, api/mpi_pack.cpp:41-660);
 *                            64-bit count, stream-ordered, device pointers.
 *   msx_reduce_tree_dev   <- the per-step MPID_Uop_call chain of the
 *                            recursive-halving/doubling schedules
 *                            (src/mpi/msmpi/mpid/reduce.cpp:3899-3989,
 *                            1088-1175) fused into one pass over p inputs.
 *
 * All functions return an MPI error class (MPI_SUCCESS = 0).  Extensions do
 * not invoke the MPI error handler; msx_last_error() describes the failure.
 */
#ifndef MSX_H_INCLUDED
#define MSX_H_INCLUDED

#include <stdint.h>
#include "mpi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* library identity */
const char* msx_version(void);
/* number of visible GPUs (0 on a host without one); never aborts */
int msx_device_count(void);
/* data plane of the collective engine for MPI_COMM_WORLD: "rccl" (RCCL
 * send/recv over xGMI, MSX_TRANSPORT=rccl and one GPU per rank), "ipc" (IPC
 * windows + remote writes) or "self" (one rank) */
const char* msx_engine_transport(void);
/* 1 when two or more ranks of MPI_COMM_WORLD run on one GPU (their PCI bus ids
 * agree), 0 when every rank has its own GPU, -1 before MPI_Init; the same on
 * every rank.  Link fractions (xGMI) mean nothing when it is 1. */
int msx_engine_gpu_shared(void);
/* phase timers of the window allreduce since the last reset (seconds):
 * out[0] stage+scatter, [1] collect wait + barrier A, [2] reduce + push,
 * [3] barrier B, [4] final collect, [5] chunks, [6] calls, [7] calls that
 * took the GPU-flag Rabenseifner schedules (two-step allreduce / reduce,
 * flag reduce_scatter); returns 8 */
int msx_engine_stats(double* out, int n, int reset);
/* link roofline probe over MPI_COMM_WORLD (collective): every rank writes
 * bytes_per_peer (capped at the window sub-slot) into each peer's window at
 * once, reps timed repetitions; *seconds = median time of one all-peer write
 * of *bytes_used per peer.  Per-GPU outbound bandwidth =
 * (size-1) * *bytes_used / *seconds. */
int msx_peer_write_bandwidth(int64_t bytes_per_peer, int reps, double* seconds, int64_t* bytes_used);
/* text of the last error raised on the calling thread ("" if none) */
const char* msx_last_error(void);

/* (op, datatype) legality exactly as the reference's check tables */
int msx_op_check(MPI_Op op, MPI_Datatype datatype);
/* element size in bytes of a predefined datatype (-1 if unknown) */
int msx_type_size(MPI_Datatype datatype);

/* The builtin op table, MPIR_Op_table (src/mpi/msmpi/mpid/op.cpp:618-622),
 * entries MPIR_Op_<op> (op.cpp:703-1923): the MPI_User_function shape that
 * MPID_Uop_call (include/op.h:171-174), the NBC reduce tasks (tasks.cpp:667,
 * 680), RMA accumulate (win.cpp:1435) and the Fortran proxy (mpif.cpp:963-976)
 * call.  Blocking: `inout` holds the result on return; operands may be device
 * memory (the gfx950 kernels run on it) or host memory (offloaded like
 * MPI_Reduce_local).  *len <= 0 does nothing.  An unsupported (op, datatype)
 * pair leaves inout untouched and sets the calling thread's op_errno to
 * MPI_ERR_OP (op.cpp:1791); a GPU failure also lands there.
 * msx_op_table(op) returns the entry of MPI_MAX .. MPI_NO_OP (NULL for any
 * other handle). */
void msx_op_max(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_min(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_sum(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_prod(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_land(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_band(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_lor(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_bor(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_lxor(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_bxor(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_minloc(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_maxloc(void* in, void* inout, int* len, MPI_Datatype* dt);
void msx_op_replace(void* in, void* inout, int* len, MPI_Datatype* dt);   /* MPIR_Op_replace op.cpp:1886 */
void msx_op_noop(void* in, void* inout, int* len, MPI_Datatype* dt);      /* MPIR_Op_noop op.cpp:1906 */
MPI_User_function* msx_op_table(MPI_Op op);
/* 1 when both operands are device memory (HBM, managed or IPC-mapped), else 0
 * (host memory, NULL, or no GPU).  The routing test of the table binding
 * (INTEGRATION.md section 2): device operands go to msx_op_table(op); host
 * operands keep the reference's own MPIR_Op_<op> loop, which beats an offload
 * below ~1 MiB (bench.py host_path.crossover).  Never initialises a GPU. */
int msx_operands_on_device(const void* in, const void* inout);
/* op_errno of the calling thread (Mpi.CallState->op_errno,
 * include/MpiCallState.h:13) and its reset (reduce.cpp:97, 3794) */
int msx_op_errno(void);
void msx_op_errno_reset(void);

/* inout[i] = inout[i] (op) in[i], i in [0,count); device pointers,
 * stream-ordered (returns after the launch, not after completion). */
int msx_reduce_local_dev(const void* in, void* inout, int64_t count,
                         MPI_Datatype datatype, MPI_Op op, void* stream);

/* packed[i*size + b] <- typed[i*extent + map(b)] for `count` instances of a
 * committed datatype (predefined or derived); typed is the buffer address the
 * type map is relative to.  Device pointers, stream-ordered. */
int msx_pack_dev(const void* typed, int64_t count, MPI_Datatype datatype, void* packed,
                 void* stream);
int msx_unpack_dev(const void* packed, int64_t count, MPI_Datatype datatype, void* typed,
                   void* stream);

/* out[i] = tree(srcs[0][i], ..., srcs[p-1][i]) with the balanced binary tree
 * ((s0 op s1) op (s2 op s3)) op ((s4 op s5) op (s6 op s7)), the left operand
 * of each combine in the reference's `inout` role.  p in {1,2,4,8,16};
 * srcs is a HOST array of device pointers; out may alias srcs[0]. */
/* SURVEY 8(e), the local reduce strong-scaled: inout[i] = inout[i] (op) in[i]
 * over one vector split into contiguous 256-byte-aligned ranges, one per GPU
 * of the node (ngpus <= 0: every visible GPU).  Host operands are pinned once
 * and each GPU combines its range in place over its own PCIe link; device
 * operands (and vectors under 1 MiB) stay on one GPU.  Blocking; MPI error
 * classes returned.  MSX_REDUCE_LOCAL_GPUS=k routes MPI_Reduce_local here. */
int msx_reduce_local_multi(const void* in, void* inout, int64_t count, MPI_Datatype datatype, MPI_Op op,
                           int ngpus);
int msx_reduce_tree_dev(const void* const* srcs, int p, void* out, int64_t count,
                        MPI_Datatype datatype, MPI_Op op, void* stream);

/* Any reference-order tree the engine evaluates: P leaves (power of two <= 16)
 * over srcs[2k] and, when bit k of pairmask is set, its fold pair srcs[2k+1]
 * (leaf k = op(srcs[2k] as inout, srcs[2k+1] as in)); leaves >= nleaves absent
 * (0 = all); or with chain != 0 the left-deep chain over srcs[0..P-1].
 * Stream-ordered, device pointers (tests and probes of the tree kernels). */
int msx_reduce_tree_spec_dev(const void* const* srcs, int P, unsigned pairmask, int nleaves, int chain,
                             void* out, int64_t count, MPI_Datatype datatype, MPI_Op op, void* stream);
/* The engine's local copy kernel (the collectives' collect step): dst <- src,
 * `bytes` bytes of device memory, stream-ordered (tests of the copy kernels). */
int msx_copy_dev(void* dst, const void* src, int64_t bytes, void* stream);
/* Test hook: pack / unpack geometry.  0 = by size (default: the one-wave tile
 * form when typed span + packed bytes exceed 512 MiB), 1 = always the
 * grid-stride form, 2 = always the tile form.  (The derived-target accumulate
 * always runs its tile form.)  The measurement kernels (HBM
 * probes, combine variants) live in the bench-only libmsx_probe.so. */
int msx_tune_pack(int mode);

/* host staging chunk size (bytes) for MPI_Reduce_local on host buffers */
int msx_set_staging_chunk(int64_t bytes);
/* host operands of MPI_Reduce_local: 0 (default) = pinned host memory is
 * combined in place by the kernel over PCIe (zero-copy), pageable memory of
 * at least 1 MiB is pinned for the call and combined
 * the same way (staged through HBM if the driver refuses to pin it);
 * 1 = every host operand is staged through HBM; 2 = pinned memory in place,
 * pageable memory staged */
int msx_set_host_mode(int mode);

/* schedule introspection for host-side tests of the collective engine
 * (mpid/reduce.cpp:3884-4066, 917-1334 restated as expression trees):
 * which = 0 allreduce tree of newrank n, 1 reduce_scatter tree of newrank n,
 * 2 pairwise chain of real rank n, 3 MPI_Reduce Rabenseifner tree of newrank n,
 * 4 MPI_Reduce binomial tree for root n.  src32[i] = real rank in kernel slot
 * i (-1 = empty). */
int msx_schedule_tree(int which, int p, int n, int* src32, int* P, unsigned* pairmask,
                      int* chain);
/* which = 0 allreduce, 1 reduce_scatter, 2 reduce: 0 recursive doubling,
 * 1 Rabenseifner, 2 recursive halving, 3 pairwise, 4 binomial */
int msx_schedule_algo(int which, int p, int64_t count, int type_size);
/* the same with the gate size taken from `dt`: MPI_Type_size (blocking calls,
 * reduce_scatter) or the extent (nbc = 1: the NBC task lists of
 * MPI_Iallreduce / MPI_Ireduce, reduce.cpp:4717,4881,6701,6740) */
int msx_schedule_algo_dt(int which, int p, int64_t count, MPI_Datatype dt, int nbc);
/* MPI_Ireduce's Rabenseifner tree of newrank n over root-relative ranks
 * (IreduceBuildScatterGatherTaskList, reduce.cpp:6267-6670) */
int msx_schedule_ireduce_tree(int p, int n, int root, int* src32, int* P, unsigned* pairmask,
                              int* chain);
int msx_schedule_newrank(int rank, int p);
/* the pipelined two-step allreduce's chunk plan for `rank` (tests): *chunk_el
 * elements per chunk; out[3i], out[3i+1], out[3i+2] = first element, end
 * element and owner newrank of each range of the rank's pieces over all
 * chunks; returns the range count, -1 if cap triples do not suffice */
int64_t msx_schedule_two_step(int p, int64_t count, int esz, int rank, int64_t* chunk_el, int64_t* out,
                              int64_t cap);
int msx_schedule_block(int p, int64_t count, int n, int64_t* start, int64_t* len);

#ifdef __cplusplus
}
#endif
#endif
