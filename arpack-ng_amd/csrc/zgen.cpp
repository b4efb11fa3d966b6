// Device operator pair of znaupd's generalized modes (bmat = 'G'): the caller's
// half of znaupd's reverse communication (SRC/znaupd.f:23-31), served on the
// GPU so the whole solve runs free (arpack_hip_znaupd_gen) instead of
// returning to the host for every OP*x and B*x:
//
//   mode 2  OP = inv[M] A,              B = M  (M Hermitian positive definite;
//                                               no x <- A x write-back)
//   mode 3  OP = inv[A - sigma M] M,    B = M  (complex sigma; at ido = 1 the
//                                               engine hands over M x, znaupd.f:60-63)
//
// The reference's drivers factor the same matrices on the host with a banded
// LU (EXAMPLES/COMPLEX/zndrv3.f: M by zgttrf; zndrv4.f: A - sigma M by zgttrf,
// solves by zgttrs).  Here the products are the complex CSR SpMV and the
// inverse is the device BiCGStab of zsolve.hip on C = A - sigma M (M itself in
// mode 2), formed once entry by entry over the union pattern in complex fp64.
#include <algorithm>
#include <utility>
#include <vector>

#include "../../include/arpack_hip.h"
#include "zgen.hpp"

namespace ahip::zdev {

namespace {
using cd = std::complex<double>;

bool download(const arpack_hip_zcsr* A, std::vector<int64_t>& rp, std::vector<int32_t>& col,
              std::vector<cd>& val) {
    int64_t n = 0, nnz = 0;
    if (arpack_hip_zcsr_info(A, &n, &nnz) != 0) return false;
    rp.resize((size_t)n + 1);
    col.resize((size_t)(nnz > 0 ? nnz : 1));
    val.resize((size_t)(nnz > 0 ? nnz : 1));
    return arpack_hip_zcsr_download(A, rp.data(), col.data(), reinterpret_cast<double*>(val.data())) == 0;
}

// C = A - sigma M entry by entry over the union of the row patterns (sorted
// copies of each row; an entry of only one matrix keeps that matrix's term)
void union_axpy(int64_t n, const std::vector<int64_t>& ap, const std::vector<int32_t>& ac,
                const std::vector<cd>& av, const std::vector<int64_t>& mp,
                const std::vector<int32_t>& mc, const std::vector<cd>& mv, cd sigma,
                std::vector<int64_t>& cp, std::vector<int32_t>& cc, std::vector<cd>& cv) {
    cp.assign((size_t)n + 1, 0);
    cc.clear();
    cv.clear();
    std::vector<std::pair<int32_t, cd>> ra, rm;
    for (int64_t i = 0; i < n; ++i) {
        ra.clear();
        rm.clear();
        for (int64_t k = ap[i]; k < ap[i + 1]; ++k) ra.push_back({ac[k], av[k]});
        for (int64_t k = mp[i]; k < mp[i + 1]; ++k) rm.push_back({mc[k], mv[k]});
        auto by_col = [](const auto& x, const auto& y) { return x.first < y.first; };
        std::stable_sort(ra.begin(), ra.end(), by_col);
        std::stable_sort(rm.begin(), rm.end(), by_col);
        size_t p = 0, q = 0;
        while (p < ra.size() || q < rm.size()) {
            if (q >= rm.size() || (p < ra.size() && ra[p].first < rm[q].first)) {
                cc.push_back(ra[p].first);
                cv.push_back(ra[p++].second);
            } else if (p >= ra.size() || rm[q].first < ra[p].first) {
                cc.push_back(rm[q].first);
                cv.push_back(-(sigma * rm[q++].second));
            } else {
                cc.push_back(ra[p].first);
                cv.push_back(ra[p++].second - sigma * rm[q++].second);
            }
        }
        cp[(size_t)i + 1] = (int64_t)cc.size();
    }
}
}  // namespace

int zgen_create(ZGen& G, const arpack_hip_zcsr* A, const arpack_hip_zcsr* M, int mode, cd sigma,
                double rtol, int maxit) {
    G = ZGen{};
    int64_t na = 0, nm = 0, nz = 0;
    if (!A || !M || mode < 2 || mode > 3 || arpack_hip_zcsr_info(A, &na, &nz) != 0 ||
        arpack_hip_zcsr_info(M, &nm, &nz) != 0 || na != nm || na <= 0)
        return -1;
    G.A = ahip_zcsr_view(A);
    G.M = ahip_zcsr_view(M);
    G.mode = mode;
    G.sigma = sigma;
    G.n = na;
    const ZCsr* solve_on = G.M;  // mode 2: inv[M]
    if (mode == 3) {
        std::vector<int64_t> ap, mp, cp;
        std::vector<int32_t> ac, mc, cc;
        std::vector<cd> av, mv, cv;
        if (!download(A, ap, ac, av) || !download(M, mp, mc, mv)) return -2;
        union_axpy(na, ap, ac, av, mp, mc, mv, sigma, cp, cc, cv);
        if (arpack_hip_zcsr_create(&G.C, na, (int64_t)cc.size(), cp.data(), cc.data(),
                                   reinterpret_cast<const double*>(cv.data())) != 0) {
            G.C = nullptr;
            return -2;
        }
        solve_on = ahip_zcsr_view(G.C);
    }
    if (zshift_create(G.S, solve_on, cd(0.0, 0.0), rtol, maxit) != 0) {
        zgen_destroy(G);
        return -2;
    }
    if (hipMalloc(&G.t, sizeof(double) * 2 * (size_t)na) != hipSuccess) {
        G.t = nullptr;
        zgen_destroy(G);
        return -2;
    }
    return 0;
}

void zgen_destroy(ZGen& G) {
    zshift_destroy(G.S);
    if (G.C) arpack_hip_zcsr_destroy(G.C);
    if (G.t) (void)hipFree(G.t);
    G = ZGen{};
}

int zgen_apply(ZGen& G, hipStream_t s, int ido, const double* x, double* y, const double* bx) {
    if (ido == 2) {  // B x = M x
        zcsr_spmv(s, *G.M, x, y);
        return hipGetLastError() == hipSuccess ? 0 : -2;
    }
    const double* rhs = G.t;
    if (G.mode == 2) {
        zcsr_spmv(s, *G.A, x, G.t);  // y = inv[M] (A x)
    } else if (ido == 1 && bx) {
        rhs = bx;                    // y = inv[A - sigma M] (M x), M x handed over
    } else {
        zcsr_spmv(s, *G.M, x, G.t);
    }
    if (hipGetLastError() != hipSuccess) return -2;
    const int it = zshift_apply(G.S, s, rhs, y, nullptr);
    return it == -2 ? -2 : it < 0 ? -1 : 0;
}

}  // namespace ahip::zdev
