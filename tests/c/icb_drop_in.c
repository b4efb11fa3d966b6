/* Drop-in check: a C caller written against the reference's ICB contract
 * (ICB/arpack.h; the pattern of TESTS/icb_arpack_c.c) compiled against
 * include/arpack_hip.h and linked with libarpack_hip.so -- no source change
 * beyond the header name.  Exit code 0 = all solves correct.  Built twice: LP64
 * against libarpack_hip.so and with -Da_int=int64_t against libarpack_hip64.so
 * (the reference's INTERFACE64 build, arpackdef.h.in:6-14).
 *   ds: dsaupd_c/dseupd_c on diag(1..N), nev 9, LM -> d = N-8 .. N
 *   dn: dnaupd_c/dneupd_c on the same diagonal
 *   zn: znaupd_c/zneupd_c on diag((k+1)(1+i)) -> d = (N-8 .. N)(1+i)
 *   ss, sn, cn: the single-precision twins (sn is TESTS/bug_1315_single.c's
 *   case, tol = 0, acceptance 0.1) */
#include <complex.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "arpack_hip.h"

#define N 1000

static void dop(const double* x, double* y) {
    for (int i = 0; i < N; ++i) y[i] = (i + 1.0) * x[i];
}
static void zop(const double _Complex* x, double _Complex* y) {
    for (int i = 0; i < N; ++i) y[i] = x[i] * ((i + 1.0) + (i + 1.0) * I);
}

static void sop(const float* x, float* y) {
    for (int i = 0; i < N; ++i) y[i] = (float)(i + 1) * x[i];
}
static void cop(const float _Complex* x, float _Complex* y) {
    for (int i = 0; i < N; ++i) y[i] = x[i] * ((float)(i + 1) + (float)(i + 1) * I);
}

static int ss(void) {
    const int nev = 9, ncv = 2 * nev + 1, lworkl = ncv * (ncv + 8);
    float *resid = calloc(N, sizeof(float)), *v = calloc(N * ncv, sizeof(float));
    float *workd = calloc(3 * N, sizeof(float)), *workl = calloc(lworkl, sizeof(float));
    float d[9], *z = calloc(N * nev, sizeof(float));
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[11], select[19];
    a_int ido = 0, info = 0;
    do {
        ssaupd_c(&ido, "I", N, "LM", nev, 1e-4f, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, &info);
        if (ido == -1 || ido == 1) sop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0 || iparam[4] < nev) return printf("ss: info %d nconv %d\n", (int)info, (int)iparam[4]), 1;
    sseupd_c(1, "A", select, d, z, N, 0.0f, "I", N, "LM", nev, 1e-4f, resid, ncv, v, N, iparam,
             ipntr, workd, workl, lworkl, &info);
    if (info < 0) return printf("ss: eupd info %d\n", (int)info), 1;
    for (int i = 0; i < nev; ++i)
        if (fabsf(d[i] - (float)(N - (nev - 1) + i)) > 1e-2f)
            return printf("ss: d[%d] = %f\n", i, d[i]), 1;
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

static int sn(void) {
    const int nev = 9, ncv = 2 * nev + 1, lworkl = 3 * ncv * ncv + 6 * ncv;
    float *resid = calloc(N, sizeof(float)), *v = calloc(N * ncv, sizeof(float));
    float *workd = calloc(3 * N, sizeof(float)), *workl = calloc(lworkl, sizeof(float));
    float dr[10], di[10], *z = calloc((N + 1) * (nev + 1), sizeof(float)), workev[3 * 19];
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[14], select[3 * 19];
    a_int ido = 0, info = 0;
    do {
        snaupd_c(&ido, "I", N, "LM", nev, 0.0f, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, &info);
        if (ido == -1 || ido == 1) sop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0) return printf("sn: info %d\n", (int)info), 1;
    sneupd_c(1, "A", select, dr, di, z, N + 1, 0.0f, 0.0f, workev, "I", N, "LM", nev, 0.0f, resid,
             ncv, v, N, iparam, ipntr, workd, workl, lworkl, &info);
    for (int i = 0; i < nev; ++i)  /* TESTS/bug_1315_single.c acceptance */
        if (fabsf(dr[i] - (float)(N - i)) > 1e-1f) return printf("sn: dr[%d] = %f\n", i, dr[i]), 1;
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

static int cn(void) {
    const int nev = 9, ncv = 2 * nev + 1, lworkl = ncv * (3 * ncv + 5);
    float _Complex *resid = calloc(N, sizeof(float _Complex));
    float _Complex *v = calloc(N * ncv, sizeof(float _Complex));
    float _Complex *workd = calloc(3 * N, sizeof(float _Complex));
    float _Complex *workl = calloc(lworkl, sizeof(float _Complex));
    float _Complex d[10], *z = calloc(N * nev, sizeof(float _Complex)), workev[2 * 19];
    float rwork[19];
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[14], select[19];
    a_int ido = 0, info = 0;
    do {
        cnaupd_c(&ido, "I", N, "LM", nev, 1e-4f, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, rwork, &info);
        if (ido == -1 || ido == 1) cop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0 || iparam[4] < nev) return printf("cn: info %d nconv %d\n", (int)info, (int)iparam[4]), 1;
    cneupd_c(1, "A", select, d, z, N, 0.0f, workev, "I", N, "LM", nev, 1e-4f, resid, ncv, v, N,
             iparam, ipntr, workd, workl, lworkl, rwork, &info);
    if (info < 0) return printf("cn: eupd info %d\n", (int)info), 1;
    for (int i = 0; i < nev; ++i) {
        int hit = 0;
        for (int k = 0; k < nev; ++k)
            hit |= fabsf(crealf(d[k]) - (float)(N - i)) < 1e-2f &&
                   fabsf(cimagf(d[k]) - (float)(N - i)) < 1e-2f;
        if (!hit) return printf("cn: %d missing\n", N - i), 1;
    }
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

static int ds(void) {
    const int nev = 9, ncv = 2 * nev + 1, lworkl = ncv * (ncv + 8);
    double *resid = calloc(N, sizeof(double)), *v = calloc(N * ncv, sizeof(double));
    double *workd = calloc(3 * N, sizeof(double)), *workl = calloc(lworkl, sizeof(double));
    double d[9], *z = calloc(N * nev, sizeof(double));
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[11], select[19];
    a_int ido = 0, info = 0;
    do {
        dsaupd_c(&ido, "I", N, "LM", nev, 1e-6, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, &info);
        if (ido == -1 || ido == 1) dop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0 || iparam[4] < nev) return printf("ds: info %d nconv %d\n", (int)info, (int)iparam[4]), 1;
    dseupd_c(1, "A", select, d, z, N, 0.0, "I", N, "LM", nev, 1e-6, resid, ncv, v, N, iparam,
             ipntr, workd, workl, lworkl, &info);
    if (info < 0) return printf("ds: eupd info %d\n", (int)info), 1;
    for (int i = 0; i < nev; ++i)
        if (fabs(d[i] - (N - (nev - 1) + i)) > 1e-5) return printf("ds: d[%d] = %f\n", i, d[i]), 1;
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

static int dn(void) {
    const int nev = 9, ncv = 2 * nev + 3, lworkl = 3 * ncv * ncv + 6 * ncv;
    double *resid = calloc(N, sizeof(double)), *v = calloc(N * ncv, sizeof(double));
    double *workd = calloc(3 * N, sizeof(double)), *workl = calloc(lworkl, sizeof(double));
    double dr[10], di[10], *z = calloc(N * (nev + 1), sizeof(double)), workev[3 * 21];
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[14], select[21];
    a_int ido = 0, info = 0;
    do {
        dnaupd_c(&ido, "I", N, "LM", nev, 1e-6, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, &info);
        if (ido == -1 || ido == 1) dop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0 || iparam[4] < nev) return printf("dn: info %d nconv %d\n", (int)info, (int)iparam[4]), 1;
    dneupd_c(1, "A", select, dr, di, z, N, 0.0, 0.0, workev, "I", N, "LM", nev, 1e-6, resid, ncv,
             v, N, iparam, ipntr, workd, workl, lworkl, &info);
    if (info < 0) return printf("dn: eupd info %d\n", (int)info), 1;
    for (int i = 0; i < nev; ++i) {  /* any order: every wanted value present */
        int hit = 0;
        for (int k = 0; k < nev; ++k) hit |= fabs(dr[k] - (N - i)) < 1e-5 && fabs(di[k]) < 1e-8;
        if (!hit) return printf("dn: %d missing\n", N - i), 1;
    }
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

static int zn(void) {
    const int nev = 9, ncv = 2 * nev + 1, lworkl = ncv * (3 * ncv + 5);
    double _Complex *resid = calloc(N, sizeof(double _Complex));
    double _Complex *v = calloc(N * ncv, sizeof(double _Complex));
    double _Complex *workd = calloc(3 * N, sizeof(double _Complex));
    double _Complex *workl = calloc(lworkl, sizeof(double _Complex));
    double _Complex d[10], *z = calloc(N * nev, sizeof(double _Complex)), workev[2 * 19];
    double rwork[19];
    a_int iparam[11] = {1, 0, 10 * N, 1, 0, 0, 1, 0, 0, 0, 0}, ipntr[14], select[19];
    a_int ido = 0, info = 0;
    do {
        znaupd_c(&ido, "I", N, "LM", nev, 1e-6, resid, ncv, v, N, iparam, ipntr, workd, workl,
                 lworkl, rwork, &info);
        if (ido == -1 || ido == 1) zop(workd + ipntr[0] - 1, workd + ipntr[1] - 1);
    } while (ido == -1 || ido == 1);
    if (info < 0 || iparam[4] < nev) return printf("zn: info %d nconv %d\n", (int)info, (int)iparam[4]), 1;
    zneupd_c(0, "A", select, d, z, N, 0.0, workev, "I", N, "LM", nev, 1e-6, resid, ncv, v, N,
             iparam, ipntr, workd, workl, lworkl, rwork, &info);
    if (info < 0) return printf("zn: eupd info %d\n", (int)info), 1;
    for (int i = 0; i < nev; ++i) {
        const double ref = N - (nev - 1) + i;
        if (fabs(creal(d[i]) - ref) > 1e-5 || fabs(cimag(d[i]) - ref) > 1e-5)
            return printf("zn: d[%d] = %f %f\n", i, creal(d[i]), cimag(d[i])), 1;
    }
    free(resid), free(v), free(workd), free(workl), free(z);
    return 0;
}

int main(void) {
    const int a = ds(), b = dn(), c = zn(), e = ss(), f = sn(), g = cn();
    a_int nopx, nbx, nrorth, nitref, nrstrt;
    float t[26];
    stat_c(&nopx, &nbx, &nrorth, &nitref, &nrstrt, t, t + 1, t + 2, t + 3, t + 4, t + 5, t + 6,
           t + 7, t + 8, t + 9, t + 10, t + 11, t + 12, t + 13, t + 14, t + 15, t + 16, t + 17,
           t + 18, t + 19, t + 20, t + 21, t + 22, t + 23, t + 24, t + 25);
    printf("ds %d dn %d zn %d ss %d sn %d cn %d (last solve: nopx %d)\n", a, b, c, e, f, g, (int)nopx);
    return a | b | c | e | f | g;
}
