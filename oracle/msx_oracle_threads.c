/*
 * msx_oracle_threads.c — the reference's collective schedules with p THREADS
 * as the p ranks (the CPU baseline of SURVEY.md §8(d) for c3-c5).
 *
 * ORACLE — TEST INFRASTRUCTURE / BENCH BASELINE ONLY.  Each thread is one rank
 * of a p-rank MS-MPI job on one host: it owns its send buffer, its receive
 * buffer and its tmp buffer, and runs the reference's step loop for its own
 * rank.  MPIC_Sendrecv becomes one memcpy from the peer's buffer into this
 * rank's tmp (the reference's shared-memory channel copies twice, sender ->
 * queue -> receiver, so this is a lower bound on its transport cost), every
 * MPID_Uop_call is oracle_reduce_local(op, dt, in=tmp, inout=mine), and a
 * barrier between steps stands for the pairwise Sendrecv synchronisation
 * (a rank reads a peer's region only after the peer finished writing it).
 *
 *   allreduce (c3, c5): MPIR_Allreduce_intra_flat, Rabenseifner branch
 *     (reduce.cpp:3927-4066; the initial copy :3814-3819), power-of-two p
 *   reduce_scatter_block (c4): MPIR_Reduce_scatter_commutative_short,
 *     recursive halving (reduce.cpp:917-1219), the branch the 32-bit nbytes
 *     gate (:1705) selects for c4's 4 GiB (the product wraps to 0)
 *
 * Same index arithmetic as msx_oracle_sched.c (whose lock-step simulation the
 * tests pin); the data each rank reads from its peer d sits at the same
 * element offsets as the region it keeps (d's send region = my receive one).
 * Buffers are first-touched by their owning thread; inputs are integer-valued
 * (fp32: i % 1021 + r, exact in any order; u64: a bit pattern per rank) and
 * the result is checked against the closed form on a strided sample.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "msx_oracle.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

typedef struct {
    int which;          /* 0 = allreduce (Rabenseifner), 1 = reduce_scatter_block (halving) */
    MPI_Op op;
    MPI_Datatype dt;
    int p;
    int64_t count;      /* allreduce: per-rank vector; reduce_scatter_block: per-rank block */
    int reps;
    int64_t esz;
    char** send;
    char** rb;
    char** tmp;
    pthread_barrier_t bar;
    double* t;          /* per rep, rank 0's clock between barriers */
    int rc;
    int bad;
} job_t;

typedef struct {
    job_t* j;
    int r;
} arg_t;

static uint64_t u64_of(int r, int64_t i)
{
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + (uint64_t)r * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 29;
    return z | (1ull << r);   /* BAND keeps the bits every rank sets */
}

static void fill(job_t* j, int r, char* buf, int64_t n)
{
    if (j->dt == MPI_FLOAT) {
        float* f = (float*)buf;
        for (int64_t i = 0; i < n; ++i) f[i] = (float)(i % 1021 + r);
    } else if (j->dt == MPI_DOUBLE) {
        double* f = (double*)buf;
        for (int64_t i = 0; i < n; ++i) f[i] = (double)((i * 7 + r * 131) % 100003);
    } else {
        uint64_t* u = (uint64_t*)buf;
        for (int64_t i = 0; i < n; ++i) u[i] = u64_of(r, i);
    }
}

/* closed form of element i (global index into the reduced vector) */
static int check(job_t* j, const char* buf, int64_t first, int64_t n)
{
    const int p = j->p;
    const int64_t stride = n > 4096 ? n / 4096 : 1;
    for (int64_t k = 0; k < n; k += stride) {
        const int64_t i = first + k;
        if (j->dt == MPI_FLOAT) {
            float want = 0.0f;
            for (int r = 0; r < p; ++r) want += (float)(i % 1021 + r);
            if (((const float*)buf)[k] != want) return 1;
        } else if (j->dt == MPI_DOUBLE) {
            double want = 0.0;
            for (int r = 0; r < p; ++r) {
                const double v = (double)((i * 7 + r * 131) % 100003);
                want = v > want ? v : want;
            }
            if (((const double*)buf)[k] != want) return 1;
        } else {
            uint64_t want = ~0ull;
            for (int r = 0; r < p; ++r) want &= u64_of(r, i);
            if (((const uint64_t*)buf)[k] != want) return 1;
        }
    }
    return 0;
}

/* Rabenseifner allreduce of rank n (= newrank, p a power of two) */
static int allreduce_rank(job_t* j, int n)
{
    const int pof2 = j->p;
    const int64_t esz = j->esz, count = j->count, bytes = count * esz;
    char* rb = j->rb[n];
    char* tmp = j->tmp[n];
    int rc = 0;
    memcpy(rb, j->send[n], (size_t)bytes);                     /* :3814-3819 */
    pthread_barrier_wait(&j->bar);
    const int64_t reduceSize = count / pof2, endSize = count % pof2;
    int send_idx = 0, recv_idx = 0, last_idx = pof2, idx_shift = pof2 >> 1;
    int mask = 1;
    while (mask < pof2) {                                        /* reduce-scatter :3941-4007 */
        const int d = n ^ mask;
        int64_t rcnt;
        if (n < d) {
            send_idx = recv_idx + idx_shift;
            rcnt = (int64_t)(send_idx - recv_idx) * reduceSize;
        } else {
            recv_idx = send_idx + idx_shift;
            rcnt = (int64_t)(last_idx - recv_idx) * reduceSize;
            if (last_idx == pof2) rcnt += endSize;
        }
        const int64_t off = reduceSize * recv_idx * esz;
        memcpy(tmp + off, j->rb[d] + off, (size_t)(rcnt * esz));
        if (rcnt) rc |= oracle_reduce_local(j->op, j->dt, tmp + off, rb + off, rcnt);
        pthread_barrier_wait(&j->bar);
        send_idx = recv_idx;
        if ((mask << 1) < pof2) {
            last_idx = recv_idx + idx_shift;
            idx_shift >>= 1;
        }
        mask <<= 1;
    }
    mask >>= 1;
    while (mask > 0) {                                           /* allgather :4010-4065 */
        const int d = n ^ mask;
        int64_t rcnt;
        if (n < d) {
            if (mask != pof2 >> 1) last_idx = last_idx + idx_shift;
            recv_idx = send_idx + idx_shift;
            rcnt = (int64_t)(last_idx - recv_idx) * reduceSize;
            if (last_idx == pof2) rcnt += endSize;
        } else {
            recv_idx = send_idx - idx_shift;
            rcnt = (int64_t)(send_idx - recv_idx) * reduceSize;
        }
        const int64_t off = reduceSize * recv_idx * esz;
        memcpy(rb + off, j->rb[d] + off, (size_t)(rcnt * esz));
        pthread_barrier_wait(&j->bar);
        if (n > d) send_idx = recv_idx;
        idx_shift <<= 1;
        mask >>= 1;
    }
    return rc;
}

/* recursive-halving reduce_scatter_block of rank n (p a power of two, equal
 * blocks of j->count): res = my send buffer's copy, tmp the receive area */
static int reduce_scatter_rank(job_t* j, int n)
{
    const int pof2 = j->p;
    const int64_t esz = j->esz, blk = j->count, bytes = blk * pof2 * esz;
    char* res = j->rb[n];
    char* tmp = j->tmp[n];
    int rc = 0;
    memcpy(res, j->send[n], (size_t)bytes);                    /* tmp_results, :998-1006 */
    pthread_barrier_wait(&j->bar);
    int send_idx = 0, recv_idx = 0, last_idx = pof2;
    for (int mask = pof2 >> 1; mask > 0; mask >>= 1) {
        const int d = n ^ mask;
        int64_t rcnt;
        if (n < d) {
            send_idx = recv_idx + mask;
            rcnt = (int64_t)(send_idx - recv_idx) * blk;
        } else {
            recv_idx = send_idx + mask;
            rcnt = (int64_t)(last_idx - recv_idx) * blk;
        }
        const int64_t off = (int64_t)recv_idx * blk * esz;
        /* tmp holds at most half the vector: the received range starts at 0 of it */
        memcpy(tmp, j->rb[d] + off, (size_t)(rcnt * esz));
        if (rcnt) rc |= oracle_reduce_local(j->op, j->dt, tmp, res + off, rcnt);
        pthread_barrier_wait(&j->bar);
        send_idx = recv_idx;
        last_idx = recv_idx + mask;
    }
    /* my block into recvbuf: the send buffer serves as recvbuf (its data was
     * copied out at the start), :1170-1180 */
    memcpy(j->send[n], res + (int64_t)n * blk * esz, (size_t)(blk * esz));
    return rc;
}

static void* rank_main(void* v)
{
    arg_t* a = (arg_t*)v;
    job_t* j = a->j;
    const int r = a->r;
    const int64_t elems = j->which == 0 ? j->count : j->count * j->p;
    const int64_t bytes = elems * j->esz;
    const int64_t tbytes = j->which == 0 ? bytes : bytes / 2 + j->esz;
    /* first touch by the owning thread (its NUMA node) */
    j->send[r] = (char*)malloc((size_t)bytes);
    j->rb[r] = (char*)malloc((size_t)bytes);
    j->tmp[r] = (char*)malloc((size_t)tbytes);
    int rc = 0;
    if (!j->send[r] || !j->rb[r] || !j->tmp[r]) rc = MPI_ERR_NO_MEM;
    else {
        memset(j->rb[r], 0, (size_t)bytes);
        memset(j->tmp[r], 0, (size_t)tbytes);
    }
    pthread_barrier_wait(&j->bar);
    if (rc == 0) {
        for (int k = 0; k < j->p; ++k)
            if (!j->send[k] || !j->rb[k] || !j->tmp[k]) rc = MPI_ERR_NO_MEM;
    }
    /* Every thread leaves the loop at the same rep: a failing call publishes
     * its error in the shared word before the closing barrier, and each thread
     * reads that word only after it (no thread writes it again before all
     * have read it), so none is left waiting at a barrier the others skip. */
    for (int rep = 0; rep < j->reps && rc == 0; ++rep) {
        fill(j, r, j->send[r], elems);                           /* outside the timed region */
        pthread_barrier_wait(&j->bar);
        const double t0 = now_s();
        const int rc1 = j->which == 0 ? allreduce_rank(j, r) : reduce_scatter_rank(j, r);
        if (rc1) __atomic_fetch_or(&j->rc, rc1, __ATOMIC_RELAXED);
        pthread_barrier_wait(&j->bar);
        if (r == 0) j->t[rep] = now_s() - t0;
        rc = __atomic_load_n(&j->rc, __ATOMIC_RELAXED);
    }
    if (rc == 0) {
        const int bad = j->which == 0 ? check(j, j->rb[r], 0, j->count)
                                      : check(j, j->send[r], (int64_t)r * j->count, j->count);
        if (bad) __atomic_fetch_add(&j->bad, 1, __ATOMIC_RELAXED);
    }
    if (rc) __atomic_fetch_or(&j->rc, rc, __ATOMIC_RELAXED);
    pthread_barrier_wait(&j->bar);
    free(j->send[r]);
    free(j->rb[r]);
    free(j->tmp[r]);
    return NULL;
}

/* Run `reps` calls of collective `which` with p threads as ranks; times[rep]
 * = seconds of call rep (all ranks between two barriers).  Returns 0 on
 * success, MPI_ERR_OTHER when the result is wrong, MPI_ERR_NO_MEM / _ARG. */
int oracle_coll_threads(int which, MPI_Op op, MPI_Datatype dt, int p, int64_t count, int reps, double* times)
{
    if (p < 1 || (p & (p - 1)) || reps < 1 || count < p || (which != 0 && which != 1)) return MPI_ERR_ARG;
    if (oracle_op_check(op, dt) != MPI_SUCCESS) return MPI_ERR_OP;
    if (dt != MPI_FLOAT && dt != MPI_DOUBLE && dt != MPI_UINT64_T) return MPI_ERR_ARG;
    job_t j;
    memset(&j, 0, sizeof(j));
    j.which = which;
    j.op = op;
    j.dt = dt;
    j.p = p;
    j.count = count;
    j.reps = reps;
    j.esz = oracle_kind_size(oracle_kind_of(dt));
    j.send = (char**)calloc((size_t)p, sizeof(char*));
    j.rb = (char**)calloc((size_t)p, sizeof(char*));
    j.tmp = (char**)calloc((size_t)p, sizeof(char*));
    j.t = times;
    pthread_barrier_init(&j.bar, NULL, (unsigned)p);
    pthread_t* th = (pthread_t*)calloc((size_t)p, sizeof(pthread_t));
    arg_t* args = (arg_t*)calloc((size_t)p, sizeof(arg_t));
    for (int r = 0; r < p; ++r) {
        args[r].j = &j;
        args[r].r = r;
        pthread_create(&th[r], NULL, rank_main, &args[r]);
    }
    for (int r = 0; r < p; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&j.bar);
    free(th);
    free(args);
    free(j.send);
    free(j.rb);
    free(j.tmp);
    if (j.rc) return j.rc == MPI_ERR_NO_MEM ? MPI_ERR_NO_MEM : MPI_ERR_OTHER;
    return j.bad ? MPI_ERR_OTHER : MPI_SUCCESS;
}
