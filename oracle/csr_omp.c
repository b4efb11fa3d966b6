/* Multithreaded CSR SpMV y = A x (fp64 values, int32 columns, int64 row pointers).
 * CPU-baseline user OP for the reference RCI loop (the user SpMV
 * must be multithreaded; SciPy's A@x is single-threaded). Test/bench
 * infrastructure only — never part of the product path. */
#include <stdint.h>
#include <omp.h>

void csr_spmv_f64(int64_t n, const int64_t *rowptr, const int32_t *col,
                  const double *val, const double *x, double *y, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double s = 0.0;
        for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) s += val[k] * x[col[k]];
        y[i] = s;
    }
}

void csr_spmv_c128(int64_t n, const int64_t *rowptr, const int32_t *col,
                   const double *val /* interleaved re,im */, const double *x,
                   double *y, int nthreads)
{
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        double sr = 0.0, si = 0.0;
        for (int64_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            double ar = val[2 * k], ai = val[2 * k + 1];
            double xr = x[2 * (int64_t)col[k]], xi = x[2 * (int64_t)col[k] + 1];
            sr += ar * xr - ai * xi;
            si += ar * xi + ai * xr;
        }
        y[2 * i] = sr;
        y[2 * i + 1] = si;
    }
}
