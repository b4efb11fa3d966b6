// Device operator pair of the generalized modes (bmat = 'G'): the caller's half
// of dsaupd's reverse communication for modes 2-5 (SRC/dsaupd.f:30-77), and of
// dnaupd's for modes 2-3 with a real shift (SRC/dnaupd.f:18-33), served on the
// GPU so the whole solve runs free (arpack_hip_dsaupd_gen /
// arpack_hip_dnaupd_gen) instead of returning to the host for every OP*x and B*x:
//
//   mode 2  OP = inv[M] A,              B = M   (x <- A x written back, dsaupd.f:40-46)
//   mode 3  OP = inv[A - sigma M] M,    B = M
//   mode 4  OP = inv[K - sigma KG] K,   B = K   (buckling: A = K, M = KG)
//   mode 5  OP = inv[A - sigma M](A + sigma M),  B = M   (Cayley)
//
// dnaupd (A nonsymmetric, M symmetric positive semi-definite):
//   mode 2  OP = inv[M] A,  B = M  (no write-back: EXAMPLES/NONSYM/dndrv3.f:215-240)
//   mode 3  OP = inv[A - sigma M] M,  B = M, sigma real (dndrv4.f:243-300);
//           C is nonsymmetric: the device BiCGStab (method kDShiftBicgstab)
//
// The products are the engine's device CSR SpMV; the inverse is a Krylov solve
// on the device (dshift.hip: CG for a positive-definite C, MINRES for an
// indefinite one) on C = A - sigma M (M itself in mode 2), formed once, exactly
// in fp64 entry by entry (a_ij - sigma m_ij, the caller's own arithmetic), as
// a CSR of the union pattern.  The reference's drivers (EXAMPLES/SYM/dsdrv3-6.f)
// factor the same C with a banded LU on the host.
#include <algorithm>
#include <cstring>
#include <vector>

#include "../../include/arpack_hip.h"
#include "dgen.hpp"
#include "zsolve.hpp"

const ahip::dev::Csr* ahip_csr_view(const arpack_hip_csr* A);  // csr.hip
const ahip::zdev::ZCsr* ahip_zcsr_view(const arpack_hip_zcsr* A);  // zsolver.cpp

namespace ahip::dev {

namespace {
// C = A - sigma B entry by entry over the union of the two row patterns (column
// order ascending within a row, as both inputs); host arrays.
void csr_axpy_host(int64_t n, const std::vector<int64_t>& ap, const std::vector<int32_t>& ac,
                   const std::vector<double>& av, const std::vector<int64_t>& bp,
                   const std::vector<int32_t>& bc, const std::vector<double>& bv, double sigma,
                   std::vector<int64_t>& cp, std::vector<int32_t>& cc, std::vector<double>& cv) {
    cp.assign((size_t)n + 1, 0);
    cc.clear();
    cv.clear();
    cc.reserve(ac.size() + bc.size());
    cv.reserve(ac.size() + bc.size());
    for (int64_t i = 0; i < n; ++i) {
        // rows may come unsorted: merge sorted copies
        std::vector<std::pair<int32_t, double>> ra, rb;
        for (int64_t k = ap[i]; k < ap[i + 1]; ++k) ra.push_back({ac[k], av[k]});
        for (int64_t k = bp[i]; k < bp[i + 1]; ++k) rb.push_back({bc[k], bv[k]});
        std::stable_sort(ra.begin(), ra.end(), [](auto& x, auto& y) { return x.first < y.first; });
        std::stable_sort(rb.begin(), rb.end(), [](auto& x, auto& y) { return x.first < y.first; });
        size_t p = 0, q = 0;
        while (p < ra.size() || q < rb.size()) {
            int32_t c;
            double v;
            if (q >= rb.size() || (p < ra.size() && ra[p].first < rb[q].first)) {
                c = ra[p].first;
                v = ra[p++].second;
            } else if (p >= ra.size() || rb[q].first < ra[p].first) {
                c = rb[q].first;
                v = -(sigma * rb[q++].second);
            } else {
                c = ra[p].first;
                v = ra[p++].second - sigma * rb[q++].second;
            }
            cc.push_back(c);
            cv.push_back(v);
        }
        cp[(size_t)i + 1] = (int64_t)cc.size();
    }
}

bool download(const arpack_hip_csr* A, std::vector<int64_t>& rp, std::vector<int32_t>& col,
              std::vector<double>& val) {
    int64_t n = 0, nnz = 0;
    if (arpack_hip_csr_info(A, &n, &nnz) != 0) return false;
    rp.resize((size_t)n + 1);
    col.resize((size_t)(nnz > 0 ? nnz : 1));
    val.resize((size_t)(nnz > 0 ? nnz : 1));
    return arpack_hip_csr_download(A, rp.data(), col.data(), val.data()) == 0;
}
}  // namespace

int dgen_create(DGen& G, const arpack_hip_csr* A, const arpack_hip_csr* B, int mode, double sigma,
                double rtol, int maxit, int method) {
    G = DGen{};
    int64_t na = 0, nb = 0, nz = 0;
    if (!A || !B || mode < 2 || mode > 5 || arpack_hip_csr_info(A, &na, &nz) != 0 ||
        arpack_hip_csr_info(B, &nb, &nz) != 0 || na != nb || na <= 0)
        return -1;
    G.A = ahip_csr_view(A);
    G.B = ahip_csr_view(B);
    G.mode = mode;
    G.sigma = sigma;
    G.n = na;
    const Csr* solve_on = G.B;  // mode 2: inv[M]
    if (mode != 2) {            // C = A - sigma M (mode 4: K - sigma KG)
        std::vector<int64_t> ap, bp, cp;
        std::vector<int32_t> ac, bc, cc;
        std::vector<double> av, bv, cv;
        if (!download(A, ap, ac, av) || !download(B, bp, bc, bv)) return -2;
        csr_axpy_host(na, ap, ac, av, bp, bc, bv, sigma, cp, cc, cv);
        if (arpack_hip_csr_create(&G.C, na, (int64_t)cc.size(), cp.data(), cc.data(), cv.data()) != 0) {
            G.C = nullptr;
            return -2;
        }
        solve_on = ahip_csr_view(G.C);
    }
    if (dshift_create(G.S, solve_on, 0.0, rtol, maxit) != 0) {
        dgen_destroy(G);
        return -2;
    }
    G.S.method = method;
    if (method == kDShiftTridiag && dshift_tridiag_factor(G.S) != 0) {  // C tridiagonal: direct
        dgen_destroy(G);
        return -1;
    }
    if (hipMalloc(&G.t, sizeof(double) * 2 * (size_t)na) != hipSuccess) {
        G.t = nullptr;
        dgen_destroy(G);
        return -2;
    }
    return 0;
}

int dgen_create_cshift(DGen& G, const arpack_hip_csr* A, const arpack_hip_csr* B, int mode,
                       double sigmar, double sigmai, double rtol, int maxit, int method) {
    G = DGen{};
    int64_t na = 0, nb = 0, nz = 0;
    if (!A || !B || (mode != 3 && mode != 4) || sigmai == 0.0 || method < 0 || method > 1 ||
        arpack_hip_csr_info(A, &na, &nz) != 0 || arpack_hip_csr_info(B, &nb, &nz) != 0 || na != nb ||
        na <= 0)
        return -1;
    G.A = ahip_csr_view(A);
    G.B = ahip_csr_view(B);
    G.mode = mode;
    G.sigma = sigmar;
    G.n = na;
    G.cshift = true;
    G.part = mode == 4 ? 1 : 0;
    // C = A - sigma M over the union pattern, in complex arithmetic (the
    // drivers' own: dndrv5.f forms A - (sigmar, sigmai) M entry by entry)
    std::vector<int64_t> ap, bp, cp;
    std::vector<int32_t> ac, bc, cc;
    std::vector<double> av, bv, cvr, cvi;
    if (!download(A, ap, ac, av) || !download(B, bp, bc, bv)) return -2;
    csr_axpy_host(na, ap, ac, av, bp, bc, bv, sigmar, cp, cc, cvr);  // re: a - sigmar m
    std::vector<double> zero(av.size(), 0.0);
    std::vector<int64_t> cp2;
    std::vector<int32_t> cc2;
    csr_axpy_host(na, ap, ac, zero, bp, bc, bv, sigmai, cp2, cc2, cvi);  // im: -sigmai m
    std::vector<double> cv(2 * cc.size());
    for (size_t k = 0; k < cc.size(); ++k) {
        cv[2 * k] = cvr[k];
        cv[2 * k + 1] = cvi[k];
    }
    if (arpack_hip_zcsr_create(&G.ZC, na, (int64_t)cc.size(), cp.data(), cc.data(), cv.data()) != 0) {
        G.ZC = nullptr;
        return -2;
    }
    G.ZS = new zdev::ZShift;
    if (zdev::zshift_create(*G.ZS, ahip_zcsr_view(G.ZC), std::complex<double>(0.0, 0.0), rtol, maxit) != 0) {
        dgen_destroy(G);
        return -2;
    }
    if (method == 1 && zdev::zshift_tridiag_factor(*G.ZS) != 0) {
        dgen_destroy(G);
        return -1;
    }
    if (hipMalloc(&G.t, sizeof(double) * 2 * (size_t)na) != hipSuccess ||
        hipMalloc(&G.zb, sizeof(double) * 4 * (size_t)na) != hipSuccess) {
        dgen_destroy(G);
        return -2;
    }
    return 0;
}

void dgen_destroy(DGen& G) {
    if (G.ZS) {
        zdev::zshift_destroy(*G.ZS);
        delete G.ZS;
    }
    if (G.ZC) arpack_hip_zcsr_destroy(G.ZC);
    if (G.zb) (void)hipFree(G.zb);
    dshift_destroy(G.S);
    if (G.C) arpack_hip_csr_destroy(G.C);
    if (G.t) (void)hipFree(G.t);
    G = DGen{};
}

// One request of the solve (ido = -1, 1 or 2, SRC/dsaupd.f:30-77): x, y,
// bx (ido = 1, modes 3-5: B x already computed by the engine) device
// pointers; xw: where mode 2 writes A x back (workd(ipntr(1))) -- dsaupd's
// contract; nullptr for dnaupd's, which has no write-back.
int dgen_apply(DGen& G, hipStream_t s, int ido, const double* x, double* y, const double* bx,
               double* xw) {
    const int64_t n = G.n;
    double* t = G.t;
    double* t2 = G.t + n;
    // B*x: the mass matrix (dsaupd's mode 4, buckling: K, the user's first
    // matrix; dnaupd's complex-shift mode 4: M)
    const Csr* bop = G.mode == 4 && !G.cshift ? G.A : G.B;
    if (ido == 2) {
        csr_spmv(s, *bop, x, y);
        return 0;
    }
    double relres = 0.0;
    const double* rhs = t;
    if (G.cshift) {  // y = Re / Im of inv[A - sigma M] (M x), M x given at ido = 1
        if (ido == 1 && bx) rhs = bx;
        else csr_spmv(s, *G.B, x, t);
        const int64_t m2 = 2 * n;
        zdev::zpack_real(s, n, rhs, G.zb);
        if (hipGetLastError() != hipSuccess) return -2;
        const int rc = zdev::zshift_apply(*G.ZS, s, G.zb, G.zb + m2, nullptr);
        if (rc == -2) return -2;
        if (rc < 0) return -1;
        zdev::zextract(s, n, G.zb + m2, G.part, y);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    switch (G.mode) {
        case 2:  // y = inv[M] (A x), and (dsaupd) x <- A x
            csr_spmv(s, *G.A, x, t);
            if (xw) copy<double>(s, n, t, xw);
            break;
        case 3:  // y = inv[A - sigma M] (M x), M x given at ido = 1
        case 4:  // y = inv[K - sigma KG] (K x), K x given at ido = 1
            if (ido == 1 && bx) rhs = bx;
            else csr_spmv(s, *bop, x, t);
            break;
        case 5:  // y = inv[A - sigma M] (A x + sigma M x)
            csr_spmv(s, *G.A, x, t);
            if (ido == 1 && bx) {
                axpby<double>(s, n, 1.0, t, G.sigma, bx);
            } else {
                csr_spmv(s, *G.B, x, t2);
                axpby<double>(s, n, 1.0, t, G.sigma, t2);
            }
            break;
        default:
            return -2;
    }
    if (hipGetLastError() != hipSuccess) return -2;
    return dshift_apply(G.S, s, rhs, y, &relres) < 0 ? -1 : 0;
}

}  // namespace ahip::dev
