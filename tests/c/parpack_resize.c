/* Two PARPACK solves in one process with different decompositions (GPU test,
 * tests/test_gpu_parpack.py::test_parpack_resize): pznaupd_c / pzneupd_c and
 * pdsaupd_c / pdseupd_c on a diagonal operator, first with 500 rows a rank,
 * then with rank 0 keeping its 500 rows while the others take 700 -- the
 * same (communicator, local rows) pair on rank 0 under a different global
 * size and row offset, which libparpack_hip.so must establish afresh at the
 * second solve's ido = 0.
 *
 * Operator: A = diag(d_g), d_g = (g + 1) (1 + 0.1 i) for global row g (real
 * case: g + 1); which = LM, nev 4, ncv 20: the wanted eigenvalues are the
 * top four d_g, known exactly.  Checks: info 0, nconv = nev, every Ritz value
 * within 1e-8 relative of its exact value, and ||A z - lambda z|| <= 1e-8 |lambda|
 * for every Ritz vector (norms summed over the ranks).  Prints "ok" on rank 0.
 *   mpiexec -n 2 oracle/_ref/tests/parpack_resize_hip
 */
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "parpack.h"

#define NEV 4
#define NCV 20

static int g_rank, g_size;

static int check_value(double complex got, double complex want, const char* what) {
    if (cabs(got - want) > 1e-8 * cabs(want)) {
        fprintf(stderr, "rank %d %s: Ritz value %.12g%+.12gi, want %.12g%+.12gi\n", g_rank, what,
                creal(got), cimag(got), creal(want), cimag(want));
        return 1;
    }
    return 0;
}

static int solve_complex(MPI_Fint fc, int nloc, long long row0, long long nglob) {
    const a_int lworkl = 3 * NCV * NCV + 5 * NCV;
    double complex *resid = calloc(nloc, sizeof(double complex)),
                   *v = calloc((size_t)nloc * NCV, sizeof(double complex)),
                   *workd = calloc(3 * (size_t)nloc, sizeof(double complex)),
                   *workl = calloc(lworkl, sizeof(double complex)),
                   *z = calloc((size_t)nloc * (NEV + 1), sizeof(double complex)),
                   *workev = calloc(2 * NCV, sizeof(double complex)), d[NEV + 1];
    double* rwork = calloc(NCV, sizeof(double));
    a_int iparam[11] = {0}, ipntr[14] = {0}, select[NCV] = {0}, ido = 0, info = 0;
    iparam[0] = 1;
    iparam[2] = 500;
    iparam[6] = 1;
    int bad = 0;
    for (;;) {
        pznaupd_c(fc, &ido, "I", nloc, "LM", NEV, 1e-10, resid, NCV, v, nloc, iparam, ipntr, workd,
                  workl, lworkl, rwork, &info);
        if (ido != -1 && ido != 1) break;
        const double complex* x = workd + ipntr[0] - 1;
        double complex* y = workd + ipntr[1] - 1;
        for (int i = 0; i < nloc; ++i) y[i] = (double)(row0 + i + 1) * (1.0 + 0.1 * I) * x[i];
    }
    if (info != 0) {
        fprintf(stderr, "rank %d pznaupd info %d\n", g_rank, (int)info);
        return 1;
    }
    pzneupd_c(fc, 1, "A", select, d, z, nloc, 0.0, workev, "I", nloc, "LM", NEV, 1e-10, resid, NCV,
              v, nloc, iparam, ipntr, workd, workl, lworkl, rwork, &info);
    if (info != 0 || iparam[4] != NEV) {
        fprintf(stderr, "rank %d pzneupd info %d nconv %d\n", g_rank, (int)info, (int)iparam[4]);
        return 1;
    }
    for (int k = 0; k < NEV; ++k) {  /* the top four, in any order */
        double complex want = (double)nglob * (1.0 + 0.1 * I);
        for (int q = 1; q < NEV; ++q) {
            const double complex c = (double)(nglob - q) * (1.0 + 0.1 * I);
            if (cabs(d[k] - c) < cabs(d[k] - want)) want = c;
        }
        bad |= check_value(d[k], want, "complex");
        double r2 = 0.0, z2 = 0.0, s[2];
        for (int i = 0; i < nloc; ++i) {
            const double complex zi = z[(size_t)k * nloc + i];
            const double complex ri = (double)(row0 + i + 1) * (1.0 + 0.1 * I) * zi - d[k] * zi;
            r2 += creal(ri * conj(ri));
            z2 += creal(zi * conj(zi));
        }
        double loc[2] = {r2, z2};
        MPI_Allreduce(loc, s, 2, MPI_DOUBLE, MPI_SUM, MPI_Comm_f2c(fc));
        if (sqrt(s[0]) > 1e-8 * cabs(d[k]) * sqrt(s[1])) {
            fprintf(stderr, "rank %d complex residual %g\n", g_rank, sqrt(s[0] / s[1]));
            bad = 1;
        }
    }
    free(resid), free(v), free(workd), free(workl), free(z), free(workev), free(rwork);
    return bad;
}

static int solve_real(MPI_Fint fc, int nloc, long long row0, long long nglob) {
    const a_int lworkl = NCV * NCV + 8 * NCV;
    double *resid = calloc(nloc, sizeof(double)), *v = calloc((size_t)nloc * NCV, sizeof(double)),
           *workd = calloc(3 * (size_t)nloc, sizeof(double)), *workl = calloc(lworkl, sizeof(double)),
           *z = calloc((size_t)nloc * NEV, sizeof(double)), d[NEV];
    a_int iparam[11] = {0}, ipntr[11] = {0}, select[NCV] = {0}, ido = 0, info = 0;
    iparam[0] = 1;
    iparam[2] = 500;
    iparam[6] = 1;
    int bad = 0;
    for (;;) {
        pdsaupd_c(fc, &ido, "I", nloc, "LM", NEV, 1e-10, resid, NCV, v, nloc, iparam, ipntr, workd,
                  workl, lworkl, &info);
        if (ido != -1 && ido != 1) break;
        const double* x = workd + ipntr[0] - 1;
        double* y = workd + ipntr[1] - 1;
        for (int i = 0; i < nloc; ++i) y[i] = (double)(row0 + i + 1) * x[i];
    }
    if (info != 0) {
        fprintf(stderr, "rank %d pdsaupd info %d\n", g_rank, (int)info);
        return 1;
    }
    pdseupd_c(fc, 1, "A", select, d, z, nloc, 0.0, "I", nloc, "LM", NEV, 1e-10, resid, NCV, v, nloc,
              iparam, ipntr, workd, workl, lworkl, &info);
    if (info != 0 || iparam[4] != NEV) {
        fprintf(stderr, "rank %d pdseupd info %d nconv %d\n", g_rank, (int)info, (int)iparam[4]);
        return 1;
    }
    for (int k = 0; k < NEV; ++k) {  /* the top four, in any order */
        double want = (double)nglob;
        for (int q = 1; q < NEV; ++q)
            if (fabs(d[k] - (double)(nglob - q)) < fabs(d[k] - want)) want = (double)(nglob - q);
        bad |= check_value(d[k], want, "real");
    }
    free(resid), free(v), free(workd), free(workl), free(z);
    return bad;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    MPI_Comm_rank(MPI_COMM_WORLD, &g_rank);
    MPI_Comm_size(MPI_COMM_WORLD, &g_size);
    const MPI_Fint fc = MPI_Comm_c2f(MPI_COMM_WORLD);
    int bad = 0;
    for (int pass = 0; pass < 2; ++pass) {
        /* pass 0: 500 rows a rank; pass 1: rank 0 keeps 500, the others 700 */
        const int nloc = pass == 0 || g_rank == 0 ? 500 : 700;
        const long long row0 = g_rank == 0 ? 0 : 500 + (long long)(g_rank - 1) * nloc;
        const long long nglob = 500 + (long long)(g_size - 1) * (pass == 0 ? 500 : 700);
        bad |= solve_complex(fc, nloc, row0, nglob);
        bad |= solve_real(fc, nloc, row0, nglob);
    }
    int any = 0;
    MPI_Allreduce(&bad, &any, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    if (g_rank == 0) printf(any ? "FAILED\n" : "ok\n");
    MPI_Finalize();
    return any ? 1 : 0;
}
