/*
 * msx_oracle_sched.c — step-by-step simulation of MS-MPI's reduction schedules.
 *
 * ORACLE — TEST INFRASTRUCTURE ONLY.  p ranks are simulated in lock step in one
 * process: every MPIC_Sendrecv of a step is a memcpy of the sender's region as
 * it stood at the start of the step, and every MPID_Uop_call is
 * oracle_reduce_local(op, dt, in=<received>, inout=<local>), with exactly the
 * buffers and index arithmetic of the reference:
 *   MPIR_Allreduce_intra_flat               reduce.cpp:3768-4104
 *   MPIR_Reduce_scatter_intra_impl          reduce.cpp:1636-1770 (32-bit nbytes gate)
 *   MPIR_Reduce_scatter_commutative_short   reduce.cpp:917-1219
 *   MPIR_Reduce_scatter_commutative_long    reduce.cpp:1225-1334
 * (the HA / node-aware variants, reduce.cpp:4180-4292, are not simulated: the
 * flat algorithm is the reference order, as with MSMPI_HA_COLLECTIVE=OFF, and
 * the one the reference takes for every message >= 256 KiB.)
 * PARITY UNPINNED: no recorded reference output covers these schedules; the
 * restatement is checked against the association orders derived from the
 * source text (tests/test_oracle.py), DESIGN.md §2.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "msx_oracle.h"

/* The flat switch points (mpid/env.cpp:514-608 via env_to_int,
 * common/mpiutil.cpp:65-91): MPICH_DEFAULT_* override the coll.h defaults;
 * unset or longer than 11 characters -> default, else the integer, >= 0. */
static uint32_t switch_point(const char* name, int defval)
{
    const char* v = getenv(name);
    if (!v || strlen(v) > 11) return (uint32_t)defval;
    long long x = strtoll(v, NULL, 10);
    if (x > 2147483647LL) x = 2147483647LL;
    if (x < 0) x = 0;
    return (uint32_t)x;
}

static int pof2_floor(int p)
{
    int v = 1;
    while (v * 2 <= p) v *= 2;
    return v;
}

typedef struct { char* buf; } rbuf;

static int combine(MPI_Op op, MPI_Datatype dt, const void* in, void* inout, int64_t n)
{
    return n > 0 ? oracle_reduce_local(op, dt, in, inout, n) : 0;
}

/* gate_size: bytes per element the algorithm gate multiplies count by --
 * MPI_Type_size for the blocking call (reduce.cpp:3821,3884), the extent for
 * the NBC task list (:4712-4717,4881). */
static int allreduce_sim(MPI_Op op, MPI_Datatype dt, int p, int64_t count,
                         const void* const* sendbufs, void* const* recvbufs, int64_t gate_size)
{
    if (oracle_op_check(op, dt) != MPI_SUCCESS) return MPI_ERR_OP;
    if (p < 1) return MPI_ERR_ARG;
    if (count == 0) return MPI_SUCCESS;
    const int64_t esz = oracle_kind_size(oracle_kind_of(dt));
    const int64_t bytes = count * esz;
    char** rb = (char**)recvbufs;
    char** tmp = (char**)calloc((size_t)p, sizeof(char*));
    char** snap = (char**)calloc((size_t)p, sizeof(char*));
    int* newrank = (int*)calloc((size_t)p, sizeof(int));
    int rc = MPI_SUCCESS;
    for (int r = 0; r < p; ++r) {
        if (sendbufs[r] != MPI_IN_PLACE) memcpy(rb[r], sendbufs[r], (size_t)bytes);  /* :3814-3819 */
        tmp[r] = (char*)malloc((size_t)bytes);
        snap[r] = (char*)malloc((size_t)bytes);
    }
    const int pof2 = pof2_floor(p), rem = p - pof2;

    /* fold (:3835-3871): even r < 2*rem sends to r+1, which combines tmp -> recvbuf */
    for (int r = 0; r < p; ++r) {
        if (r < 2 * rem) {
            if ((r & 1) == 0) {
                newrank[r] = -1;
            } else {
                memcpy(tmp[r], rb[r - 1], (size_t)bytes);
                rc |= combine(op, dt, tmp[r], rb[r], count);
                newrank[r] = r / 2;
            }
        } else {
            newrank[r] = r - rem;
        }
    }
    int* real = (int*)calloc((size_t)pof2, sizeof(int));
    for (int r = 0; r < p; ++r) if (newrank[r] >= 0) real[newrank[r]] = r;

    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)gate_size);   /* :3884 / :4881 */
    if (nbytes <= switch_point("MPICH_DEFAULT_ALLREDUCE_SHORT_MSG", 262144) || count < pof2) {
        /* recursive doubling (:3890-3926): commutative builtin -> Uop(tmp, recvbuf) */
        for (int mask = 1; mask < pof2; mask <<= 1) {
            for (int n = 0; n < pof2; ++n) memcpy(snap[real[n]], rb[real[n]], (size_t)bytes);
            for (int n = 0; n < pof2; ++n) {
                const int r = real[n], dst = real[n ^ mask];
                memcpy(tmp[r], snap[dst], (size_t)bytes);
                rc |= combine(op, dt, tmp[r], rb[r], count);
            }
        }
    } else {
        /* reduce-scatter + allgather (:3927-4066) */
        const int64_t reduceSize = count / pof2, endSize = count % pof2;
        int *send_idx = calloc((size_t)pof2, sizeof(int)), *recv_idx = calloc((size_t)pof2, sizeof(int));
        int *last_idx = calloc((size_t)pof2, sizeof(int)), *idx_shift = calloc((size_t)pof2, sizeof(int));
        int64_t *scnt = calloc((size_t)pof2, sizeof(int64_t)), *rcnt = calloc((size_t)pof2, sizeof(int64_t));
        for (int n = 0; n < pof2; ++n) { last_idx[n] = pof2; idx_shift[n] = pof2 >> 1; }
        int mask = 1;
        while (mask < pof2) {
            for (int n = 0; n < pof2; ++n) {
                const int nd = n ^ mask;
                if (n < nd) {
                    send_idx[n] = recv_idx[n] + idx_shift[n];
                    rcnt[n] = (int64_t)(send_idx[n] - recv_idx[n]) * reduceSize;
                    scnt[n] = (int64_t)(last_idx[n] - send_idx[n]) * reduceSize;
                    if (last_idx[n] == pof2) scnt[n] += endSize;
                } else {
                    recv_idx[n] = send_idx[n] + idx_shift[n];
                    scnt[n] = (int64_t)(recv_idx[n] - send_idx[n]) * reduceSize;
                    rcnt[n] = (int64_t)(last_idx[n] - recv_idx[n]) * reduceSize;
                    if (last_idx[n] == pof2) rcnt[n] += endSize;
                }
            }
            for (int n = 0; n < pof2; ++n) memcpy(snap[real[n]], rb[real[n]], (size_t)bytes);
            for (int n = 0; n < pof2; ++n) {
                const int r = real[n], d = n ^ mask;
                const int64_t off = reduceSize * recv_idx[n] * esz;
                /* what d sends: its send region, which is our recv region */
                memcpy(tmp[r] + off, snap[real[d]] + reduceSize * send_idx[d] * esz, (size_t)(rcnt[n] * esz));
                rc |= combine(op, dt, tmp[r] + off, rb[r] + off, rcnt[n]);
            }
            for (int n = 0; n < pof2; ++n) {
                send_idx[n] = recv_idx[n];
                if ((mask << 1) < pof2) {
                    last_idx[n] = recv_idx[n] + idx_shift[n];
                    idx_shift[n] >>= 1;
                }
            }
            mask <<= 1;
        }
        mask >>= 1;
        while (mask > 0) {
            for (int n = 0; n < pof2; ++n) {
                const int nd = n ^ mask;
                if (n < nd) {
                    if (mask != pof2 >> 1) last_idx[n] = last_idx[n] + idx_shift[n];
                    recv_idx[n] = send_idx[n] + idx_shift[n];
                    scnt[n] = (int64_t)(recv_idx[n] - send_idx[n]) * reduceSize;
                    rcnt[n] = (int64_t)(last_idx[n] - recv_idx[n]) * reduceSize;
                    if (last_idx[n] == pof2) rcnt[n] += endSize;
                } else {
                    recv_idx[n] = send_idx[n] - idx_shift[n];
                    rcnt[n] = (int64_t)(send_idx[n] - recv_idx[n]) * reduceSize;
                    scnt[n] = (int64_t)(last_idx[n] - send_idx[n]) * reduceSize;
                    if (last_idx[n] == pof2) scnt[n] += endSize;
                }
            }
            for (int n = 0; n < pof2; ++n) memcpy(snap[real[n]], rb[real[n]], (size_t)bytes);
            for (int n = 0; n < pof2; ++n) {
                const int r = real[n], d = n ^ mask;
                memcpy(rb[r] + reduceSize * recv_idx[n] * esz,
                       snap[real[d]] + reduceSize * send_idx[d] * esz, (size_t)(rcnt[n] * esz));
            }
            for (int n = 0; n < pof2; ++n) {
                if (n > (n ^ mask)) send_idx[n] = recv_idx[n];
                idx_shift[n] <<= 1;
            }
            mask >>= 1;
        }
        free(send_idx); free(recv_idx); free(last_idx); free(idx_shift); free(scnt); free(rcnt);
    }
    /* unfold (:4071-4092) */
    for (int r = 0; r < 2 * rem; r += 2) memcpy(rb[r], rb[r + 1], (size_t)bytes);

    for (int r = 0; r < p; ++r) { free(tmp[r]); free(snap[r]); }
    free(tmp); free(snap); free(newrank); free(real);
    return rc ? MPI_ERR_OP : MPI_SUCCESS;
}

int oracle_allreduce(MPI_Op op, MPI_Datatype dt, int p, int64_t count,
                     const void* const* sendbufs, void* const* recvbufs)
{
    return allreduce_sim(op, dt, p, count, sendbufs, recvbufs, oracle_type_size(dt));
}

/* IallreduceBuildTaskList (reduce.cpp:4699-4982): fold, recursive doubling
 * (IallreduceBuildRecursiveDoublingTaskList :4601-4693) or reduce-scatter +
 * allgather (IallreduceBuildReduceScatterAllGatherTaskList :4346-4595) with
 * the blocking call's peers, index arithmetic and -- builtin ops being
 * commutative -- NbcTask::ExecuteReduce's Uop(recv, reduce) roles
 * (tasks.cpp:680-686); only the gate differs: fullExtent = extent * count. */
int oracle_iallreduce(MPI_Op op, MPI_Datatype dt, int p, int64_t count,
                      const void* const* sendbufs, void* const* recvbufs)
{
    return allreduce_sim(op, dt, p, count, sendbufs, recvbufs, oracle_kind_size(oracle_kind_of(dt)));
}

int oracle_reduce_scatter(MPI_Op op, MPI_Datatype dt, int p, const int* recvcounts,
                          const void* const* sendbufs, void* const* recvbufs)
{
    if (oracle_op_check(op, dt) != MPI_SUCCESS) return MPI_ERR_OP;
    const int64_t esz = oracle_kind_size(oracle_kind_of(dt));
    int64_t* disps = (int64_t*)calloc((size_t)p + 1, sizeof(int64_t));
    for (int i = 0; i < p; ++i) disps[i + 1] = disps[i] + recvcounts[i];
    const int64_t total = disps[p];
    int rc = MPI_SUCCESS;
    if (total == 0) { free(disps); return MPI_SUCCESS; }
    const int64_t bytes = total * esz;
    /* :1705 nbytes = (unsigned)(total_count * type_size).  MPI_Ireduce_scatter
     * takes this same simulation: IreduceScatterBuildTaskList gates on the
     * same product (cbBuffer, :3201 -- type size, unlike the allreduce /
     * reduce NBC gates), its short list (:1987-2406) has the blocking fold,
     * newcnts/newdisps merge, BinomialChildBuilderDescending = mask pof2/2..1
     * (tasks.h:448-469), TrimmedToOriginalRankOdd = newdst*2+1 / newdst+rem
     * (:1975-1981) and keep-lower-half rule, and its long list (:2412-2676)
     * walks src = rank-1, rank-2, ... like the blocking pairwise loop; for
     * the (commutative) builtin ops NbcTask::ExecuteReduce ignores rightOrder
     * and calls Uop(recv, reduce) (tasks.cpp:665-686), the blocking roles. */
    const uint32_t nbytes = (uint32_t)((uint64_t)total * (uint64_t)oracle_type_size(dt));
    char** res = (char**)calloc((size_t)p, sizeof(char*));
    char** tmp = (char**)calloc((size_t)p, sizeof(char*));
    char** snap = (char**)calloc((size_t)p, sizeof(char*));
    for (int r = 0; r < p; ++r) {
        res[r] = (char*)malloc((size_t)bytes);
        tmp[r] = (char*)malloc((size_t)bytes);
        snap[r] = (char*)malloc((size_t)bytes);
        const void* src = sendbufs[r] != MPI_IN_PLACE ? sendbufs[r] : recvbufs[r];
        memcpy(res[r], src, (size_t)bytes);
    }
    if (nbytes < switch_point("MPICH_DEFAULT_REDSCAT_COMMUTATIVE_LONG_MSG", 524288)) {
        /* recursive halving (:917-1219) */
        const int pof2 = pof2_floor(p), rem = p - pof2;
        int* newrank = (int*)calloc((size_t)p, sizeof(int));
        int* real = (int*)calloc((size_t)pof2, sizeof(int));
        for (int r = 0; r < p; ++r) {
            if (r < 2 * rem) {
                if ((r & 1) == 0) newrank[r] = -1;
                else {
                    memcpy(tmp[r], res[r - 1], (size_t)bytes);
                    rc |= combine(op, dt, tmp[r], res[r], total);
                    newrank[r] = r / 2;
                }
            } else newrank[r] = r - rem;
            if (newrank[r] >= 0) real[newrank[r]] = r;
        }
        int64_t* newcnts = (int64_t*)calloc((size_t)pof2, sizeof(int64_t));
        int64_t* newdisps = (int64_t*)calloc((size_t)pof2 + 1, sizeof(int64_t));
        {
            int i = 0, old_i = 0;
            for (i = 0; i < rem; i++) {
                newcnts[i] = recvcounts[old_i] + recvcounts[old_i + 1];
                old_i += 2;
                newdisps[i + 1] = newdisps[i] + newcnts[i];
            }
            for (; old_i < p; ++old_i, ++i) {
                newcnts[i] = recvcounts[old_i];
                newdisps[i + 1] = newdisps[i] + newcnts[i];
            }
        }
        int *send_idx = calloc((size_t)pof2, sizeof(int)), *recv_idx = calloc((size_t)pof2, sizeof(int));
        int *last_idx = calloc((size_t)pof2, sizeof(int));
        int64_t* rcnt = calloc((size_t)pof2, sizeof(int64_t));
        for (int n = 0; n < pof2; ++n) last_idx[n] = pof2;
        for (int mask = pof2 >> 1; mask > 0; mask >>= 1) {
            for (int n = 0; n < pof2; ++n) {
                const int nd = n ^ mask;
                rcnt[n] = 0;
                if (n < nd) {
                    send_idx[n] = recv_idx[n] + mask;
                    for (int i = recv_idx[n]; i < send_idx[n]; i++) rcnt[n] += newcnts[i];
                } else {
                    recv_idx[n] = send_idx[n] + mask;
                    for (int i = recv_idx[n]; i < last_idx[n]; i++) rcnt[n] += newcnts[i];
                }
            }
            for (int n = 0; n < pof2; ++n) memcpy(snap[real[n]], res[real[n]], (size_t)bytes);
            for (int n = 0; n < pof2; ++n) {
                const int r = real[n], d = n ^ mask;
                if (rcnt[n]) {
                    const int64_t off = newdisps[recv_idx[n]] * esz;
                    memcpy(tmp[r] + off, snap[real[d]] + newdisps[send_idx[d]] * esz, (size_t)(rcnt[n] * esz));
                    rc |= combine(op, dt, tmp[r] + off, res[r] + off, rcnt[n]);
                }
            }
            for (int n = 0; n < pof2; ++n) {
                send_idx[n] = recv_idx[n];
                last_idx[n] = recv_idx[n] + mask;
            }
        }
        for (int r = 0; r < p; ++r) {
            if (newrank[r] >= 0 && recvcounts[r])
                memcpy(recvbufs[r], res[r] + disps[r] * esz, (size_t)recvcounts[r] * esz);
        }
        for (int r = 0; r < 2 * rem; r += 2)   /* odd sends the even rank's block */
            if (recvcounts[r]) memcpy(recvbufs[r], res[r + 1] + disps[r] * esz, (size_t)recvcounts[r] * esz);
        free(newrank); free(real); free(newcnts); free(newdisps);
        free(send_idx); free(recv_idx); free(last_idx); free(rcnt);
    } else {
        /* pairwise exchange (:1225-1334): recvbuf = own block, then p-1 combines */
        for (int r = 0; r < p; ++r) {
            const int64_t n = recvcounts[r];
            char* acc = (char*)malloc((size_t)(n * esz) + 1);
            memcpy(acc, res[r] + disps[r] * esz, (size_t)(n * esz));
            int src = r;
            for (int i = p - 1; i > 0; i--) {
                if (--src < 0) src += p;
                rc |= combine(op, dt, res[src] + disps[r] * esz, acc, n);
            }
            if (n) memcpy(recvbufs[r], acc, (size_t)(n * esz));
            free(acc);
        }
    }
    for (int r = 0; r < p; ++r) { free(res[r]); free(tmp[r]); free(snap[r]); }
    free(res); free(tmp); free(snap); free(disps);
    return rc ? MPI_ERR_OP : MPI_SUCCESS;
}

/* MPIR_Reduce_intra_flat (reduce.cpp:63-566), commutative builtin ops.
 * Rabenseifner (bytes > 64 KiB, count >= pof2): ODD ranks < 2*rem fold into
 * the even rank below (:136-165), recursive halving as in allreduce (with
 * real rank = newdst < rem ? 2*newdst : newdst + rem), then a gather to root
 * that only moves data (:330-450): root's block j is the value its owner
 * computed.  Binomial (otherwise, :489-537): relative ranks to root, node
 * relrank receives from relrank|mask and combines Uop(tmp=received, recvbuf). */
static int reduce_sim(MPI_Op op, MPI_Datatype dt, int p, int root, int64_t count,
                      const void* const* sendbufs, void* recvbuf_root, int64_t gate_size, int relative)
{
    if (oracle_op_check(op, dt) != MPI_SUCCESS) return MPI_ERR_OP;
    if (p < 1 || root < 0 || root >= p) return MPI_ERR_ARG;
    if (count == 0) return MPI_SUCCESS;
    const int64_t esz = oracle_kind_size(oracle_kind_of(dt));
    const int64_t bytes = count * esz;
    char** rb = (char**)calloc((size_t)p, sizeof(char*));
    char** tmp = (char**)calloc((size_t)p, sizeof(char*));
    char** snap = (char**)calloc((size_t)p, sizeof(char*));
    int rc = 0;
    for (int r = 0; r < p; ++r) {
        rb[r] = (char*)malloc((size_t)bytes);
        tmp[r] = (char*)malloc((size_t)bytes);
        snap[r] = (char*)malloc((size_t)bytes);
        memcpy(rb[r], sendbufs[r], (size_t)bytes);
    }
    const int pof2 = pof2_floor(p), rem = p - pof2;
    const uint32_t nbytes = (uint32_t)((uint64_t)count * (uint64_t)gate_size);   /* :151 / :6740 */
    /* absolute rank of (relative) rank q: the blocking call works on absolute
     * ranks, the NBC scatter-gather on ranks relative to the root (:6309,
     * :6471 RankAdd(TrimmedToOriginalRankEven(rem, peer), root)) */
    const int base = relative ? root : 0;
#define ABS_RANK(q) (((q) + base) % p)
    if (nbytes > switch_point("MPICH_DEFAULT_REDUCE_SHORT_MSG", 65536) && count >= pof2) {
        int* real = (int*)calloc((size_t)pof2, sizeof(int));
        for (int q = 0; q < p; ++q) {
            const int r = ABS_RANK(q);
            if (q < 2 * rem) {
                if ((q & 1) == 0) {                 /* even: receive from q+1 and combine (:190-203, :6386-6420) */
                    memcpy(tmp[r], rb[ABS_RANK(q + 1)], (size_t)bytes);
                    rc |= combine(op, dt, tmp[r], rb[r], count);
                    real[q / 2] = r;
                }
            } else {
                real[q - rem] = r;
            }
        }
#undef ABS_RANK
        const int64_t reduceSize = count / pof2, endSize = count % pof2;
        int *send_idx = calloc((size_t)pof2, sizeof(int)), *recv_idx = calloc((size_t)pof2, sizeof(int));
        int *last_idx = calloc((size_t)pof2, sizeof(int)), *idx_shift = calloc((size_t)pof2, sizeof(int));
        int64_t* rcnt = calloc((size_t)pof2, sizeof(int64_t));
        for (int n = 0; n < pof2; ++n) { last_idx[n] = pof2; idx_shift[n] = pof2 >> 1; }
        for (int mask = 1; mask < pof2; mask <<= 1) {
            for (int n = 0; n < pof2; ++n) {
                const int nd = n ^ mask;
                if (n < nd) {
                    send_idx[n] = recv_idx[n] + idx_shift[n];
                    rcnt[n] = (int64_t)(send_idx[n] - recv_idx[n]) * reduceSize;
                } else {
                    recv_idx[n] = send_idx[n] + idx_shift[n];
                    rcnt[n] = (int64_t)(last_idx[n] - recv_idx[n]) * reduceSize;
                    if (last_idx[n] == pof2) rcnt[n] += endSize;
                }
            }
            for (int n = 0; n < pof2; ++n) memcpy(snap[real[n]], rb[real[n]], (size_t)bytes);
            for (int n = 0; n < pof2; ++n) {
                const int r = real[n], d = n ^ mask;
                const int64_t off = reduceSize * recv_idx[n] * esz;
                memcpy(tmp[r] + off, snap[real[d]] + reduceSize * send_idx[d] * esz, (size_t)(rcnt[n] * esz));
                rc |= combine(op, dt, tmp[r] + off, rb[r] + off, rcnt[n]);
            }
            for (int n = 0; n < pof2; ++n) {
                send_idx[n] = recv_idx[n];
                if ((mask << 1) < pof2) {
                    last_idx[n] = recv_idx[n] + idx_shift[n];
                    idx_shift[n] >>= 1;
                }
            }
        }
        /* gather: block j lives at newrank bitrev(j) after the halving */
        int bits = 0;
        while ((1 << bits) < pof2) ++bits;
        char* out = (char*)recvbuf_root;
        for (int j = 0; j < pof2; ++j) {
            int o = 0;
            for (int b = 0; b < bits; ++b) o |= ((j >> b) & 1) << (bits - 1 - b);
            const int64_t lo = (int64_t)j * reduceSize, ln = reduceSize + (j == pof2 - 1 ? endSize : 0);
            memcpy(out + lo * esz, rb[real[o]] + lo * esz, (size_t)(ln * esz));
        }
        free(real); free(send_idx); free(recv_idx); free(last_idx); free(idx_shift); free(rcnt);
    } else {
        /* binomial (:489-537), commutative: lroot = root */
        for (int mask = 1; mask < p; mask <<= 1) {
            for (int r = 0; r < p; ++r) memcpy(snap[r], rb[r], (size_t)bytes);
            for (int r = 0; r < p; ++r) {
                int rel = r - root;
                if (rel < 0) rel += p;
                if ((rel & (mask - 1)) != 0) continue;          /* already sent and left */
                if ((rel & mask) == 0) {
                    int src = rel | mask;
                    if (src < p) {
                        src = (src + root) % p;
                        memcpy(tmp[r], snap[src], (size_t)bytes);
                        rc |= combine(op, dt, tmp[r], rb[r], count);
                    }
                }
            }
        }
        memcpy(recvbuf_root, rb[root], (size_t)bytes);
    }
    for (int r = 0; r < p; ++r) { free(rb[r]); free(tmp[r]); free(snap[r]); }
    free(rb); free(tmp); free(snap);
    return rc ? MPI_ERR_OP : MPI_SUCCESS;
}

int oracle_reduce(MPI_Op op, MPI_Datatype dt, int p, int root, int64_t count,
                  const void* const* sendbufs, void* recvbuf_root)
{
    return reduce_sim(op, dt, p, root, count, sendbufs, recvbuf_root, oracle_type_size(dt), 0);
}

/* IreduceBuildTaskList (reduce.cpp:6676-6768): extent gate (:6701, :6740);
 * IreduceBuildScatterGatherTaskList over root-relative ranks, the even
 * relative rank combining Uop(tmp = x_{rel+1}, recvbuf) (:6403-6411,
 * rightOrder false, commutative builtin -> tasks.cpp:680-686), recursive
 * halving with ascending offsets keeping the lower half (:6461-6559), gather
 * by translated rank (:6570-6664: scatter rank s holds chunk bitrev(s));
 * IreduceBuildBinomialTaskList (:6005-6198): children rank+1, +2, +4 ...
 * combined in that order, Uop(tmp, recvbuf) -- the blocking binomial tree. */
int oracle_ireduce(MPI_Op op, MPI_Datatype dt, int p, int root, int64_t count,
                   const void* const* sendbufs, void* recvbuf_root)
{
    return reduce_sim(op, dt, p, root, count, sendbufs, recvbuf_root, oracle_kind_size(oracle_kind_of(dt)), 1);
}

/* MPI_Scan / MPI_Exscan as the reference runs them: the NBC task lists of
 * IscanBuildTaskList (reduce.cpp:5285-5576) and IexscanBuildTaskList
 * (:5671-5960) executed by NbcTask::ExecuteScan (tasks.cpp:694-766).
 * partial = x_r (and recvbuf = x_r for Scan); for mask = 1, 2, ...:
 * dst = r ^ mask (< p); the last step only goes from the lower to the higher
 * rank.  rank > dst: Uop(tmp, partial); Uop(tmp, recvbuf), or recvbuf = tmp on
 * Exscan's first such step (copyOnly).  rank < dst: Uop(tmp, partial).
 * Exscan leaves rank 0's recvbuf untouched (undefined). */
int oracle_scan(MPI_Op op, MPI_Datatype dt, int p, int64_t count, int exclusive,
                const void* const* sendbufs, void* const* recvbufs)
{
    if (oracle_op_check(op, dt) != MPI_SUCCESS) return MPI_ERR_OP;
    if (count == 0 || p < 1) return MPI_SUCCESS;
    const int64_t esz = oracle_kind_size(oracle_kind_of(dt));
    const int64_t bytes = count * esz;
    char** part = (char**)calloc((size_t)p, sizeof(char*));
    char** snap = (char**)calloc((size_t)p, sizeof(char*));
    char* tmp = (char*)malloc((size_t)bytes);
    int* have = (int*)calloc((size_t)p, sizeof(int));
    int rc = 0;
    for (int r = 0; r < p; ++r) {
        part[r] = (char*)malloc((size_t)bytes);
        snap[r] = (char*)malloc((size_t)bytes);
        memcpy(part[r], sendbufs[r], (size_t)bytes);
        if (!exclusive) { memcpy(recvbufs[r], sendbufs[r], (size_t)bytes); have[r] = 1; }
    }
    for (int mask = 1; mask < p; mask <<= 1) {
        const int last = (mask << 1) >= p;
        for (int r = 0; r < p; ++r) memcpy(snap[r], part[r], (size_t)bytes);
        for (int r = 0; r < p; ++r) {
            const int dst = r ^ mask;
            if (dst >= p || (last && r < dst)) continue;
            memcpy(tmp, snap[dst], (size_t)bytes);
            rc |= combine(op, dt, tmp, part[r], count);
            if (r > dst) {
                if (exclusive && !have[r]) { memcpy(recvbufs[r], tmp, (size_t)bytes); have[r] = 1; }
                else rc |= combine(op, dt, tmp, recvbufs[r], count);
            }
        }
    }
    for (int r = 0; r < p; ++r) { free(part[r]); free(snap[r]); }
    free(part); free(snap); free(tmp); free(have);
    return rc ? MPI_ERR_OP : MPI_SUCCESS;
}
