/*
 * reduce_local_demo.c — a plain C MPI program built against include/mpi.h and
 * linked with libmsmpi_mi355x.so, unchanged from what it would be against
 * MS-MPI (BASELINE.json configs[0]: MPI_Reduce_local MPI_SUM MPI_INT, 1 MiB).
 *
 *   gcc -O2 -I include examples/reduce_local_demo.c \
 *       -L microsoft-mpi_amd/lib -lmsmpi_mi355x -Wl,-rpath,$PWD/microsoft-mpi_amd/lib
 *
 * Checks the result against the C loop of the reference (op.cpp:42-52, int
 * wrap-around) and prints "OK <checksum>"; exits with the MPI error class on
 * failure (no GPU: the library reports "no usable MI355X" and aborts).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mpi.h"

int main(int argc, char** argv)
{
    MPI_Init(&argc, &argv);
    const int n = (1 << 20) / (int)sizeof(int);
    int* in = malloc((size_t)n * sizeof(int));
    int* inout = malloc((size_t)n * sizeof(int));
    int* expect = malloc((size_t)n * sizeof(int));
    uint32_t x = 12345u;
    for (int i = 0; i < n; ++i) {
        x = x * 1664525u + 1013904223u;
        in[i] = (int)x;
        x = x * 1664525u + 1013904223u;
        inout[i] = (int)x;
        expect[i] = (int)((uint32_t)inout[i] + (uint32_t)in[i]);   /* two's-complement wrap */
    }
    int rc = MPI_Reduce_local(in, inout, n, MPI_INT, MPI_SUM);
    if (rc != MPI_SUCCESS) {
        fprintf(stderr, "MPI_Reduce_local failed: %d\n", rc);
        return rc;
    }
    if (memcmp(inout, expect, (size_t)n * sizeof(int)) != 0) {
        fprintf(stderr, "result mismatch\n");
        return 1;
    }
    uint64_t sum = 0;
    for (int i = 0; i < n; ++i) sum += (uint32_t)inout[i];
    int size = 0, rank = 0;
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    /* a one-rank MPI_Allreduce of the same data is a copy */
    int* out = malloc((size_t)n * sizeof(int));
    rc = MPI_Allreduce(inout, out, n, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (rc != MPI_SUCCESS || (size == 1 && memcmp(out, inout, (size_t)n * sizeof(int)) != 0)) {
        fprintf(stderr, "MPI_Allreduce failed: %d\n", rc);
        return rc ? rc : 1;
    }
    printf("OK %llu rank %d of %d\n", (unsigned long long)sum, rank, size);
    free(in); free(inout); free(expect); free(out);
    MPI_Finalize();
    return 0;
}
