/*
 * collectives_demo.c — an ordinary MPI program (plain C, gcc) on host
 * buffers, linked against libmsmpi_mi355x.so: the reduction collectives,
 * a user-defined op, a non-blocking allreduce, a derived datatype with
 * MPI_Pack, and one-sided accumulate under fence and under passive locks.
 * Every expected value is computed here exactly (integer data).
 *
 *   gcc -O2 -I include examples/collectives_demo.c -L microsoft-mpi_amd/lib \
 *       -lmsmpi_mi355x -Wl,-rpath,$PWD/microsoft-mpi_amd/lib -o collectives_demo
 *   MSX_SIZE=2 MSX_RANK=r MSX_BOOTSTRAP_ADDR=127.0.0.1 MSX_BOOTSTRAP_PORT=P ./collectives_demo
 *
 * Exit status 0 when every check passed on this rank.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static int fails = 0;

static void check(int ok, const char* what, int rank)
{
    if (!ok) {
        ++fails;
        fprintf(stderr, "rank %d: FAILED %s\n", rank, what);
    }
}

/* inout = max(inout, in) + 1: commutative, not associative (order-revealing) */
static void max_plus_one(void* in, void* inout, int* len, MPI_Datatype* dt)
{
    const int* a = (const int*)in;
    int* b = (int*)inout;
    (void)dt;
    for (int i = 0; i < *len; ++i) b[i] = (a[i] > b[i] ? a[i] : b[i]) + 1;
}

int main(int argc, char** argv)
{
    int rank, p;
    MPI_Init(&argc, &argv);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &p);
    MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);

    enum { N = 100003 };
    int* x = malloc(sizeof(int) * N);
    int* y = malloc(sizeof(int) * N * (p > 0 ? p : 1));
    double* d = malloc(sizeof(double) * N);
    double* e = malloc(sizeof(double) * N);
    int ok;

    /* MPI_Allreduce SUM, in place */
    for (int i = 0; i < N; ++i) x[i] = i * 3 + rank * 1000;
    ok = MPI_Allreduce(MPI_IN_PLACE, x, N, MPI_INT, MPI_SUM, MPI_COMM_WORLD) == MPI_SUCCESS;
    for (int i = 0; ok && i < N; ++i) ok = x[i] == p * i * 3 + 1000 * (p * (p - 1) / 2);
    check(ok, "allreduce SUM in place", rank);

    /* MPI_Reduce MAX of doubles to the last rank */
    for (int i = 0; i < N; ++i) d[i] = (double)((i * 7 + rank * 13) % 1009) - 500.25;
    ok = MPI_Reduce(d, e, N, MPI_DOUBLE, MPI_MAX, p - 1, MPI_COMM_WORLD) == MPI_SUCCESS;
    if (rank == p - 1)
        for (int i = 0; ok && i < N; ++i) {
            double m = -1e300;
            for (int r = 0; r < p; ++r) {
                const double v = (double)((i * 7 + r * 13) % 1009) - 500.25;
                if (v > m) m = v;
            }
            ok = e[i] == m;
        }
    check(ok, "reduce MAX double", rank);

    /* MPI_Reduce_scatter_block BXOR, N elements per rank */
    for (int i = 0; i < N * p; ++i) y[i] = (i * 2654435761u) ^ (unsigned)(rank * 40503);
    ok = MPI_Reduce_scatter_block(y, x, N, MPI_INT, MPI_BXOR, MPI_COMM_WORLD) == MPI_SUCCESS;
    for (int i = 0; ok && i < N; ++i) {
        unsigned v = 0;
        for (int r = 0; r < p; ++r) v ^= ((unsigned)(rank * N + i) * 2654435761u) ^ (unsigned)(r * 40503);
        ok = (unsigned)x[i] == v;
    }
    check(ok, "reduce_scatter_block BXOR", rank);

    /* MPI_Scan SUM */
    for (int i = 0; i < N; ++i) x[i] = (rank + 1) * (i % 97);
    ok = MPI_Scan(x, y, N, MPI_INT, MPI_SUM, MPI_COMM_WORLD) == MPI_SUCCESS;
    for (int i = 0; ok && i < N; ++i) ok = y[i] == (i % 97) * (rank + 1) * (rank + 2) / 2;
    check(ok, "scan SUM", rank);

    /* a user-defined op (p <= 2 has a closed form for the non-associative op) */
    MPI_Op op;
    MPI_Op_create(max_plus_one, 1, &op);
    for (int i = 0; i < N; ++i) x[i] = i + 10 * rank;
    ok = MPI_Allreduce(x, y, N, MPI_INT, op, MPI_COMM_WORLD) == MPI_SUCCESS;
    if (p <= 2)
        for (int i = 0; ok && i < N; ++i) ok = y[i] == (p == 1 ? i : i + 11);
    check(ok, "allreduce with a user op", rank);
    MPI_Op_free(&op);

    /* MPI_Iallreduce + MPI_Wait (completes in the engine's worker) */
    MPI_Request req;
    for (int i = 0; i < N; ++i) x[i] = ~(1 << ((i + rank) % 31));
    ok = MPI_Iallreduce(x, y, N, MPI_INT, MPI_BAND, MPI_COMM_WORLD, &req) == MPI_SUCCESS;
    ok = ok && MPI_Wait(&req, MPI_STATUS_IGNORE) == MPI_SUCCESS;
    for (int i = 0; ok && i < N; ++i) {
        int v = -1;
        for (int r = 0; r < p; ++r) v &= ~(1 << ((i + r) % 31));
        ok = y[i] == v;
    }
    check(ok, "iallreduce BAND + wait", rank);

    /* a derived datatype: MPI_Pack of vector(100, 2, 5) of MPI_INT */
    MPI_Datatype vec;
    MPI_Type_vector(100, 2, 5, MPI_INT, &vec);
    MPI_Type_commit(&vec);
    for (int i = 0; i < 500; ++i) x[i] = i * 11 + rank;
    int pos = 0;
    ok = MPI_Pack(x, 1, vec, y, 4096, &pos, MPI_COMM_WORLD) == MPI_SUCCESS && pos == 800;
    for (int k = 0; ok && k < 100; ++k) ok = y[2 * k] == x[5 * k] && y[2 * k + 1] == x[5 * k + 1];
    check(ok, "MPI_Pack of a vector type", rank);
    MPI_Type_free(&vec);

    /* one-sided: fence accumulate into the next rank, then a passive-target
       fetch-and-add on rank 0 */
    int* wbuf = calloc(1024, sizeof(int));
    MPI_Win win;
    ok = MPI_Win_create(wbuf, 1024 * sizeof(int), sizeof(int), MPI_INFO_NULL, MPI_COMM_WORLD, &win) == MPI_SUCCESS;
    for (int i = 0; i < 512; ++i) x[i] = rank * 100 + i;
    ok = ok && MPI_Win_fence(0, win) == MPI_SUCCESS;
    ok = ok && MPI_Accumulate(x, 512, MPI_INT, (rank + 1) % p, 0, 512, MPI_INT, MPI_SUM, win) == MPI_SUCCESS;
    ok = ok && MPI_Win_fence(0, win) == MPI_SUCCESS;
    const int prev = (rank + p - 1) % p;
    for (int i = 0; ok && i < 512; ++i) ok = wbuf[i] == prev * 100 + i;
    check(ok, "fence accumulate", rank);
    int one = 1, ticket = -1;
    ok = MPI_Win_lock(MPI_LOCK_SHARED, 0, 0, win) == MPI_SUCCESS;
    ok = ok && MPI_Fetch_and_op(&one, &ticket, MPI_INT, 0, 1000, MPI_SUM, win) == MPI_SUCCESS;
    ok = ok && MPI_Win_unlock(0, win) == MPI_SUCCESS;
    ok = ok && ticket >= 0 && ticket < p;
    MPI_Barrier(MPI_COMM_WORLD);
    if (rank == 0) ok = ok && wbuf[1000] == p;
    check(ok, "passive fetch-and-op", rank);
    MPI_Win_free(&win);
    free(wbuf);

    printf("collectives_demo rank %d of %d: %s\n", rank, p, fails ? "FAILED" : "OK");
    free(x);
    free(y);
    free(d);
    free(e);
    MPI_Finalize();
    return fails ? 1 : 0;
}
