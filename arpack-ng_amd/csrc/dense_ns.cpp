// Host small-dense kit of the NONSYMMETRIC Arnoldi cycle (dnaupd family):
// the ncv x ncv upper-Hessenberg work that the reference hands to LAPACK
// (dlahqr, dtrevc, dlanv2, dlaln2, dladiv, dlanhs) and ARPACK's own helpers
// (dsortc, dngets, dnconv, dneigh, the bulge chase of dnapps).  Restated from
// the published LAPACK >= 3.10 algorithms; CPU-tested bit for bit against the
// image's LAPACK and the reference's internal routines (tests/test_kit_ns.py).
//
// Column-major, 0-based, `ld` = leading dimension.  H(i,j) below is written
// with the reference's 1-based indices through the accessor macros.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "dense.hpp"

namespace ahip::la {

namespace {
inline double sgn(double a, double b) { return std::signbit(b) ? -std::fabs(a) : std::fabs(a); }
constexpr double kUlp = DBL_EPSILON;  // dlamch('P') = eps * base
// Level-1 BLAS the reference's LAPACK calls, with the arithmetic of the
// image's OpenBLAS x86-64 kernels (fused multiply-add; verified bitwise in
// tests/test_kit_ns.py): drot and daxpy.
inline double rot_x(double c, double s, double x, double y) { return std::fma(c, x, s * y); }
inline double rot_y(double c, double s, double x, double y) { return std::fma(c, y, -(s * x)); }
inline void axpy(int n, double a, const double* x, double* y) {
    if (a == 0.0) return;
    for (int q = 0; q < n; ++q) y[q] = std::fma(a, x[q], y[q]);
}
}  // namespace

// ---------------------------------------------------------------- dlanv2 ----
void lanv2(double& a, double& b, double& c, double& d, double& rt1r, double& rt1i, double& rt2r,
           double& rt2i, double& cs, double& sn) {
    const double multpl = 4.0;
    const double safmin = kSafmin, eps = kUlp;
    const double safmn2 = std::pow(2.0, (int)(std::log(safmin / eps) / std::log(2.0) / 2.0));
    const double safmx2 = 1.0 / safmn2;
    if (c == 0.0) {
        cs = 1.0;
        sn = 0.0;
    } else if (b == 0.0) {
        cs = 0.0;
        sn = 1.0;
        const double temp = d;
        d = a;
        a = temp;
        b = -c;
        c = 0.0;
    } else if ((a - d) == 0.0 && sgn(1.0, b) != sgn(1.0, c)) {
        cs = 1.0;
        sn = 0.0;
    } else {
        double temp = a - d;
        double p = 0.5 * temp;
        const double bcmax = std::max(std::fabs(b), std::fabs(c));
        const double bcmis = std::min(std::fabs(b), std::fabs(c)) * sgn(1.0, b) * sgn(1.0, c);
        double scale = std::max(std::fabs(p), bcmax);
        double z = (p / scale) * p + (bcmax / scale) * bcmis;
        if (z >= multpl * eps) {  // real eigenvalues
            z = p + sgn(std::sqrt(scale) * std::sqrt(z), p);
            a = d + z;
            d = d - (bcmax / z) * bcmis;
            const double tau = lapy2(c, z);
            cs = z / tau;
            sn = c / tau;
            b = b - c;
            c = 0.0;
        } else {  // complex or almost equal real eigenvalues: equalise the diagonal
            int count = 0;
            double sigma = b + c;
            for (;;) {
                ++count;
                scale = std::max(std::fabs(temp), std::fabs(sigma));
                if (scale >= safmx2) {
                    sigma *= safmn2;
                    temp *= safmn2;
                    if (count <= 20) continue;
                }
                if (scale <= safmn2) {
                    sigma *= safmx2;
                    temp *= safmx2;
                    if (count <= 20) continue;
                }
                break;
            }
            p = 0.5 * temp;
            double tau = lapy2(sigma, temp);
            cs = std::sqrt(0.5 * (1.0 + std::fabs(sigma) / tau));
            sn = -(p / (tau * cs)) * sgn(1.0, sigma);
            const double aa = a * cs + b * sn, bb = -a * sn + b * cs;
            const double cc = c * cs + d * sn, dd = -c * sn + d * cs;
            a = aa * cs + cc * sn;
            b = bb * cs + dd * sn;
            c = -aa * sn + cc * cs;
            d = -bb * sn + dd * cs;
            temp = 0.5 * (a + d);
            a = temp;
            d = temp;
            if (c != 0.0) {
                if (b != 0.0) {
                    if (sgn(1.0, b) == sgn(1.0, c)) {  // real: reduce to upper triangular
                        const double sab = std::sqrt(std::fabs(b)), sac = std::sqrt(std::fabs(c));
                        p = sgn(sab * sac, c);
                        tau = 1.0 / std::sqrt(std::fabs(b + c));
                        a = temp + p;
                        d = temp - p;
                        b = b - c;
                        c = 0.0;
                        const double cs1 = sab * tau, sn1 = sac * tau;
                        temp = cs * cs1 - sn * sn1;
                        sn = cs * sn1 + sn * cs1;
                        cs = temp;
                    }
                } else {
                    b = -c;
                    c = 0.0;
                    temp = cs;
                    cs = -sn;
                    sn = temp;
                }
            }
        }
    }
    rt1r = a;
    rt2r = d;
    if (c == 0.0) {
        rt1i = 0.0;
        rt2i = 0.0;
    } else {
        rt1i = std::sqrt(std::fabs(b)) * std::sqrt(std::fabs(c));
        rt2i = -rt1i;
    }
}

// ---------------------------------------------------------------- dlanhs ----
double lanhs1(int n, const double* a, int lda) {  // norm '1'
    double value = 0.0;
    for (int j = 0; j < n; ++j) {
        double sum = 0.0;
        for (int i = 0; i <= std::min(n - 1, j + 1); ++i) sum += std::fabs(a[i + (size_t)j * lda]);
        if (value < sum || std::isnan(sum)) value = sum;
    }
    return value;
}

// ---------------------------------------------------------------- dlahqr ----
// Double-shift QR on H(ilo:ihi, ilo:ihi) (1-based bounds), LAPACK 3.10+
// (Ahues-Kressner deflation, exceptional shifts every KEXSH=10 iterations
// without deflation).  z: rows iloz..ihiz, leading dimension ldz.
int lahqr(bool wantt, bool wantz, int n, int ilo, int ihi, double* h, int ldh, double* wr,
          double* wi, int iloz, int ihiz, double* z, int ldz) {
#define H(i, j) h[((i)-1) + (size_t)((j)-1) * ldh]
#define Z(i, j) z[((i)-1) + (size_t)((j)-1) * ldz]
    const double dat1 = 3.0 / 4.0, dat2 = -0.4375;
    const int kexsh = 10;
    if (n == 0) return 0;
    if (ilo == ihi) {
        wr[ilo - 1] = H(ilo, ilo);
        wi[ilo - 1] = 0.0;
        return 0;
    }
    for (int j = ilo; j <= ihi - 3; ++j) {
        H(j + 2, j) = 0.0;
        H(j + 3, j) = 0.0;
    }
    if (ilo <= ihi - 2) H(ihi, ihi - 2) = 0.0;
    const int nh = ihi - ilo + 1;
    const int nz = ihiz - iloz + 1;
    const double safmin = kSafmin;
    const double ulp = kUlp;
    const double smlnum = safmin * ((double)nh / ulp);
    int i1 = 1, i2 = n;
    if (wantt) {
        i1 = 1;
        i2 = n;
    }
    const int itmax = 30 * std::max(10, nh);
    int kdefl = 0;
    int i = ihi;
    double v[3];
    for (;;) {  // label 20
        int l = ilo;
        if (i < ilo) return 0;
        bool converged = false;
        for (int its = 0; its <= itmax; ++its) {
            int k;
            for (k = i; k >= l + 1; --k) {
                if (std::fabs(H(k, k - 1)) <= smlnum) break;
                double tst = std::fabs(H(k - 1, k - 1)) + std::fabs(H(k, k));
                if (tst == 0.0) {
                    if (k - 2 >= ilo) tst = tst + std::fabs(H(k - 1, k - 2));
                    if (k + 1 <= ihi) tst = tst + std::fabs(H(k + 1, k));
                }
                if (std::fabs(H(k, k - 1)) <= ulp * tst) {
                    const double ab = std::max(std::fabs(H(k, k - 1)), std::fabs(H(k - 1, k)));
                    const double ba = std::min(std::fabs(H(k, k - 1)), std::fabs(H(k - 1, k)));
                    const double aa = std::max(std::fabs(H(k, k)), std::fabs(H(k - 1, k - 1) - H(k, k)));
                    const double bb = std::min(std::fabs(H(k, k)), std::fabs(H(k - 1, k - 1) - H(k, k)));
                    const double s = aa + ab;
                    if (ba * (ab / s) <= std::max(smlnum, ulp * (bb * (aa / s)))) break;
                }
            }
            l = k;
            if (l > ilo) H(l, l - 1) = 0.0;
            if (l >= i - 1) {
                converged = true;
                break;
            }
            ++kdefl;
            if (!wantt) {
                i1 = l;
                i2 = i;
            }
            double h11, h12, h21, h22;
            if (kdefl % (2 * kexsh) == 0) {
                const double s = std::fabs(H(i, i - 1)) + std::fabs(H(i - 1, i - 2));
                h11 = dat1 * s + H(i, i);
                h12 = dat2 * s;
                h21 = s;
                h22 = h11;
            } else if (kdefl % kexsh == 0) {
                const double s = std::fabs(H(l + 1, l)) + std::fabs(H(l + 2, l + 1));
                h11 = dat1 * s + H(l, l);
                h12 = dat2 * s;
                h21 = s;
                h22 = h11;
            } else {
                h11 = H(i - 1, i - 1);
                h21 = H(i, i - 1);
                h12 = H(i - 1, i);
                h22 = H(i, i);
            }
            double s = std::fabs(h11) + std::fabs(h12) + std::fabs(h21) + std::fabs(h22);
            double rt1r, rt1i, rt2r, rt2i;
            if (s == 0.0) {
                rt1r = rt1i = rt2r = rt2i = 0.0;
            } else {
                h11 /= s;
                h21 /= s;
                h12 /= s;
                h22 /= s;
                const double tr = (h11 + h22) / 2.0;
                const double det = (h11 - tr) * (h22 - tr) - h12 * h21;
                const double rtdisc = std::sqrt(std::fabs(det));
                if (det >= 0.0) {
                    rt1r = tr * s;
                    rt2r = rt1r;
                    rt1i = rtdisc * s;
                    rt2i = -rt1i;
                } else {
                    rt1r = tr + rtdisc;
                    rt2r = tr - rtdisc;
                    if (std::fabs(rt1r - h22) <= std::fabs(rt2r - h22)) {
                        rt1r = rt1r * s;
                        rt2r = rt1r;
                    } else {
                        rt2r = rt2r * s;
                        rt1r = rt2r;
                    }
                    rt1i = rt2i = 0.0;
                }
            }
            int m;
            for (m = i - 2; m >= l; --m) {
                double h21s = H(m + 1, m);
                s = std::fabs(H(m, m) - rt2r) + std::fabs(rt2i) + std::fabs(h21s);
                h21s = H(m + 1, m) / s;
                v[0] = h21s * H(m, m + 1) + (H(m, m) - rt1r) * ((H(m, m) - rt2r) / s) - rt1i * (rt2i / s);
                v[1] = h21s * (H(m, m) + H(m + 1, m + 1) - rt1r - rt2r);
                v[2] = h21s * H(m + 2, m + 1);
                s = std::fabs(v[0]) + std::fabs(v[1]) + std::fabs(v[2]);
                v[0] /= s;
                v[1] /= s;
                v[2] /= s;
                if (m == l) break;
                const double h00 = std::fabs(H(m, m - 1)) * (std::fabs(v[1]) + std::fabs(v[2]));
                const double h01 = ulp * std::fabs(v[0]) *
                                   (std::fabs(H(m - 1, m - 1)) + std::fabs(H(m, m)) + std::fabs(H(m + 1, m + 1)));
                if (h00 <= h01) break;
            }
            for (int kk = m; kk <= i - 1; ++kk) {
                const int nr = std::min(3, i - kk + 1);
                if (kk > m) std::memcpy(v, &H(kk, kk - 1), sizeof(double) * nr);
                double t1;
                larfg(nr, v[0], v + 1, 1, t1);
                if (kk > m) {
                    H(kk, kk - 1) = v[0];
                    H(kk + 1, kk - 1) = 0.0;
                    if (kk < i - 1) H(kk + 2, kk - 1) = 0.0;
                } else if (m > l) {
                    H(kk, kk - 1) = H(kk, kk - 1) * (1.0 - t1);
                }
                const double v2 = v[1], t2 = t1 * v2;
                if (nr == 3) {
                    const double v3 = v[2], t3 = t1 * v3;
                    for (int j = kk; j <= i2; ++j) {
                        const double sum = H(kk, j) + v2 * H(kk + 1, j) + v3 * H(kk + 2, j);
                        H(kk, j) = H(kk, j) - sum * t1;
                        H(kk + 1, j) = H(kk + 1, j) - sum * t2;
                        H(kk + 2, j) = H(kk + 2, j) - sum * t3;
                    }
                    for (int j = i1; j <= std::min(kk + 3, i); ++j) {
                        const double sum = H(j, kk) + v2 * H(j, kk + 1) + v3 * H(j, kk + 2);
                        H(j, kk) = H(j, kk) - sum * t1;
                        H(j, kk + 1) = H(j, kk + 1) - sum * t2;
                        H(j, kk + 2) = H(j, kk + 2) - sum * t3;
                    }
                    if (wantz) {
                        for (int j = iloz; j <= ihiz; ++j) {
                            const double sum = Z(j, kk) + v2 * Z(j, kk + 1) + v3 * Z(j, kk + 2);
                            Z(j, kk) = Z(j, kk) - sum * t1;
                            Z(j, kk + 1) = Z(j, kk + 1) - sum * t2;
                            Z(j, kk + 2) = Z(j, kk + 2) - sum * t3;
                        }
                    }
                } else if (nr == 2) {
                    for (int j = kk; j <= i2; ++j) {
                        const double sum = H(kk, j) + v2 * H(kk + 1, j);
                        H(kk, j) = H(kk, j) - sum * t1;
                        H(kk + 1, j) = H(kk + 1, j) - sum * t2;
                    }
                    for (int j = i1; j <= i; ++j) {
                        const double sum = H(j, kk) + v2 * H(j, kk + 1);
                        H(j, kk) = H(j, kk) - sum * t1;
                        H(j, kk + 1) = H(j, kk + 1) - sum * t2;
                    }
                    if (wantz) {
                        for (int j = iloz; j <= ihiz; ++j) {
                            const double sum = Z(j, kk) + v2 * Z(j, kk + 1);
                            Z(j, kk) = Z(j, kk) - sum * t1;
                            Z(j, kk + 1) = Z(j, kk + 1) - sum * t2;
                        }
                    }
                }
            }
        }
        if (!converged) return i;  // failure to converge
        if (l == i) {
            wr[i - 1] = H(i, i);
            wi[i - 1] = 0.0;
        } else if (l == i - 1) {
            double cs, sn;
            lanv2(H(i - 1, i - 1), H(i - 1, i), H(i, i - 1), H(i, i), wr[i - 2], wi[i - 2], wr[i - 1],
                  wi[i - 1], cs, sn);
            if (wantt) {
                if (i2 > i)  // drot on rows i-1, i, columns i+1..i2
                    for (int j = i + 1; j <= i2; ++j) {
                        const double x = H(i - 1, j), y = H(i, j);
                        H(i - 1, j) = rot_x(cs, sn, x, y);
                        H(i, j) = rot_y(cs, sn, x, y);
                    }
                for (int j = i1; j <= i - 2; ++j) {  // columns i-1, i, rows i1..i-2
                    const double x = H(j, i - 1), y = H(j, i);
                    H(j, i - 1) = rot_x(cs, sn, x, y);
                    H(j, i) = rot_y(cs, sn, x, y);
                }
            }
            if (wantz) {
                for (int j = iloz; j < iloz + nz; ++j) {
                    const double x = Z(j, i - 1), y = Z(j, i);
                    Z(j, i - 1) = rot_x(cs, sn, x, y);
                    Z(j, i) = rot_y(cs, sn, x, y);
                }
            }
        }
        kdefl = 0;
        i = l - 1;
    }
#undef H
#undef Z
}

// ---------------------------------------------------------------- dladiv ----
namespace {
double ladiv2(double a, double b, double c, double d, double r, double t) {
    if (r != 0.0) {
        const double br = b * r;
        if (br != 0.0) return (a + br) * t;
        return a * t + (b * t) * r;
    }
    return (a + d * (b / c)) * t;
}
void ladiv1(double a, double b, double c, double d, double& p, double& q) {
    const double r = d / c;
    const double t = 1.0 / (c + d * r);
    p = ladiv2(a, b, c, d, r, t);
    a = -a;
    q = ladiv2(b, a, c, d, r, t);
}
}  // namespace

void ladiv(double a, double b, double c, double d, double& p, double& q) {
    double aa = a, bb = b, cc = c, dd = d;
    double ab = std::max(std::fabs(a), std::fabs(b));
    double cd = std::max(std::fabs(c), std::fabs(d));
    double s = 1.0;
    const double ov = DBL_MAX, un = kSafmin, eps = kEps, bs = 2.0;
    const double be = bs / (eps * eps);
    if (ab >= 0.5 * ov) {
        aa *= 0.5;
        bb *= 0.5;
        s *= 2.0;
    }
    if (cd >= 0.5 * ov) {
        cc *= 0.5;
        dd *= 0.5;
        s *= 0.5;
    }
    if (ab <= un * bs / eps) {
        aa *= be;
        bb *= be;
        s /= be;
    }
    if (cd <= un * bs / eps) {
        cc *= be;
        dd *= be;
        s *= be;
    }
    if (std::fabs(d) <= std::fabs(c)) {
        ladiv1(aa, bb, cc, dd, p, q);
    } else {
        ladiv1(bb, aa, dd, cc, p, q);
        q = -q;
    }
    p *= s;
    q *= s;
}

// ---------------------------------------------------------------- dlaln2 ----
// Solves (ca*A - w*D) X = s*B (ltrans = false only; A is na x na, na in {1,2};
// w = wr + i*wi complex when nw = 2).  x(ldx, nw).
int laln2(int na, int nw, double smin, double ca, const double* a, int lda, double d1, double d2,
          const double* b, int ldb, double wr, double wi, double* x, int ldx, double& scale,
          double& xnorm) {
    static const bool zswap[4] = {false, false, true, true};
    static const bool rswap[4] = {false, true, false, true};
    static const int ipivot[4][4] = {{1, 2, 3, 4}, {2, 1, 4, 3}, {3, 4, 1, 2}, {4, 3, 2, 1}};
#define A(i, j) a[((i)-1) + (size_t)((j)-1) * lda]
#define B(i, j) b[((i)-1) + (size_t)((j)-1) * ldb]
#define X(i, j) x[((i)-1) + (size_t)((j)-1) * ldx]
    const double smlnum = 2.0 * kSafmin;
    const double bignum = 1.0 / smlnum;
    const double smini = std::max(smin, smlnum);
    int info = 0;
    scale = 1.0;
    if (na == 1) {
        if (nw == 1) {
            double csr = ca * A(1, 1) - wr * d1;
            double cnorm = std::fabs(csr);
            if (cnorm < smini) {
                csr = smini;
                cnorm = smini;
                info = 1;
            }
            const double bnorm = std::fabs(B(1, 1));
            if (cnorm < 1.0 && bnorm > 1.0) {
                if (bnorm > bignum * cnorm) scale = 1.0 / bnorm;
            }
            X(1, 1) = (B(1, 1) * scale) / csr;
            xnorm = std::fabs(X(1, 1));
        } else {
            double csr = ca * A(1, 1) - wr * d1;
            double csi = -wi * d1;
            double cnorm = std::fabs(csr) + std::fabs(csi);
            if (cnorm < smini) {
                csr = smini;
                csi = 0.0;
                cnorm = smini;
                info = 1;
            }
            const double bnorm = std::fabs(B(1, 1)) + std::fabs(B(1, 2));
            if (cnorm < 1.0 && bnorm > 1.0) {
                if (bnorm > bignum * cnorm) scale = 1.0 / bnorm;
            }
            ladiv(scale * B(1, 1), scale * B(1, 2), csr, csi, X(1, 1), X(1, 2));
            xnorm = std::fabs(X(1, 1)) + std::fabs(X(1, 2));
        }
        return info;
    }
    double crv[4], civ[4];  // CR / CI column-major: (1,1),(2,1),(1,2),(2,2)
    crv[0] = ca * A(1, 1) - wr * d1;
    crv[3] = ca * A(2, 2) - wr * d2;
    crv[1] = ca * A(2, 1);
    crv[2] = ca * A(1, 2);
    if (nw == 1) {
        double cmax = 0.0;
        int icmax = 0;
        for (int j = 1; j <= 4; ++j)
            if (std::fabs(crv[j - 1]) > cmax) {
                cmax = std::fabs(crv[j - 1]);
                icmax = j;
            }
        if (cmax < smini) {
            const double bnorm = std::max(std::fabs(B(1, 1)), std::fabs(B(2, 1)));
            if (smini < 1.0 && bnorm > 1.0) {
                if (bnorm > bignum * smini) scale = 1.0 / bnorm;
            }
            const double temp = scale / smini;
            X(1, 1) = temp * B(1, 1);
            X(2, 1) = temp * B(2, 1);
            xnorm = temp * bnorm;
            return 1;
        }
        const double ur11 = crv[icmax - 1];
        const double cr21 = crv[ipivot[icmax - 1][1] - 1];
        const double ur12 = crv[ipivot[icmax - 1][2] - 1];
        const double cr22 = crv[ipivot[icmax - 1][3] - 1];
        const double ur11r = 1.0 / ur11;
        const double lr21 = ur11r * cr21;
        double ur22 = cr22 - ur12 * lr21;
        if (std::fabs(ur22) < smini) {
            ur22 = smini;
            info = 1;
        }
        double br1, br2;
        if (rswap[icmax - 1]) {
            br1 = B(2, 1);
            br2 = B(1, 1);
        } else {
            br1 = B(1, 1);
            br2 = B(2, 1);
        }
        br2 = br2 - lr21 * br1;
        const double bbnd = std::max(std::fabs(br1 * (ur22 * ur11r)), std::fabs(br2));
        if (bbnd > 1.0 && std::fabs(ur22) < 1.0) {
            if (bbnd >= bignum * std::fabs(ur22)) scale = 1.0 / bbnd;
        }
        const double xr2 = (br2 * scale) / ur22;
        const double xr1 = (scale * br1) * ur11r - xr2 * (ur11r * ur12);
        if (zswap[icmax - 1]) {
            X(1, 1) = xr2;
            X(2, 1) = xr1;
        } else {
            X(1, 1) = xr1;
            X(2, 1) = xr2;
        }
        xnorm = std::max(std::fabs(xr1), std::fabs(xr2));
        if (xnorm > 1.0 && cmax > 1.0) {
            if (xnorm > bignum / cmax) {
                const double temp = cmax / bignum;
                X(1, 1) = temp * X(1, 1);
                X(2, 1) = temp * X(2, 1);
                xnorm = temp * xnorm;
                scale = temp * scale;
            }
        }
        return info;
    }
    civ[0] = -wi * d1;
    civ[1] = 0.0;
    civ[2] = 0.0;
    civ[3] = -wi * d2;
    double cmax = 0.0;
    int icmax = 0;
    for (int j = 1; j <= 4; ++j)
        if (std::fabs(crv[j - 1]) + std::fabs(civ[j - 1]) > cmax) {
            cmax = std::fabs(crv[j - 1]) + std::fabs(civ[j - 1]);
            icmax = j;
        }
    if (cmax < smini) {
        const double bnorm = std::max(std::fabs(B(1, 1)) + std::fabs(B(1, 2)),
                                      std::fabs(B(2, 1)) + std::fabs(B(2, 2)));
        if (smini < 1.0 && bnorm > 1.0) {
            if (bnorm > bignum * smini) scale = 1.0 / bnorm;
        }
        const double temp = scale / smini;
        X(1, 1) = temp * B(1, 1);
        X(2, 1) = temp * B(2, 1);
        X(1, 2) = temp * B(1, 2);
        X(2, 2) = temp * B(2, 2);
        xnorm = temp * bnorm;
        return 1;
    }
    const double ur11 = crv[icmax - 1], ui11 = civ[icmax - 1];
    const double cr21 = crv[ipivot[icmax - 1][1] - 1], ci21 = civ[ipivot[icmax - 1][1] - 1];
    const double ur12 = crv[ipivot[icmax - 1][2] - 1], ui12 = civ[ipivot[icmax - 1][2] - 1];
    const double cr22 = crv[ipivot[icmax - 1][3] - 1], ci22 = civ[ipivot[icmax - 1][3] - 1];
    double ur11r, ui11r, lr21, li21, ur12s, ui12s, ur22, ui22;
    if (icmax == 1 || icmax == 4) {
        if (std::fabs(ur11) > std::fabs(ui11)) {
            const double temp = ui11 / ur11;
            ur11r = 1.0 / (ur11 * (1.0 + temp * temp));
            ui11r = -temp * ur11r;
        } else {
            const double temp = ur11 / ui11;
            ui11r = -1.0 / (ui11 * (1.0 + temp * temp));
            ur11r = -temp * ui11r;
        }
        lr21 = cr21 * ur11r;
        li21 = cr21 * ui11r;
        ur12s = ur12 * ur11r;
        ui12s = ur12 * ui11r;
        ur22 = cr22 - ur12 * lr21;
        ui22 = ci22 - ur12 * li21;
    } else {
        ur11r = 1.0 / ur11;
        ui11r = 0.0;
        lr21 = cr21 * ur11r;
        li21 = ci21 * ur11r;
        ur12s = ur12 * ur11r;
        ui12s = ui12 * ur11r;
        ur22 = cr22 - ur12 * lr21 + ui12 * li21;
        ui22 = -ur12 * li21 - ui12 * lr21;
    }
    const double u22abs = std::fabs(ur22) + std::fabs(ui22);
    if (u22abs < smini) {
        ur22 = smini;
        ui22 = 0.0;
        info = 1;
    }
    double br1, br2, bi1, bi2;
    if (rswap[icmax - 1]) {
        br2 = B(1, 1);
        br1 = B(2, 1);
        bi2 = B(1, 2);
        bi1 = B(2, 2);
    } else {
        br1 = B(1, 1);
        br2 = B(2, 1);
        bi1 = B(1, 2);
        bi2 = B(2, 2);
    }
    br2 = br2 - lr21 * br1 + li21 * bi1;
    bi2 = bi2 - li21 * br1 - lr21 * bi1;
    const double bbnd = std::max((std::fabs(br1) + std::fabs(bi1)) *
                                     (u22abs * (std::fabs(ur11r) + std::fabs(ui11r))),
                                 std::fabs(br2) + std::fabs(bi2));
    if (bbnd > 1.0 && u22abs < 1.0) {
        if (bbnd >= bignum * u22abs) {
            scale = 1.0 / bbnd;
            br1 *= scale;
            bi1 *= scale;
            br2 *= scale;
            bi2 *= scale;
        }
    }
    double xr2, xi2;
    ladiv(br2, bi2, ur22, ui22, xr2, xi2);
    const double xr1 = ur11r * br1 - ui11r * bi1 - ur12s * xr2 + ui12s * xi2;
    const double xi1 = ui11r * br1 + ur11r * bi1 - ui12s * xr2 - ur12s * xi2;
    if (zswap[icmax - 1]) {
        X(1, 1) = xr2;
        X(2, 1) = xr1;
        X(1, 2) = xi2;
        X(2, 2) = xi1;
    } else {
        X(1, 1) = xr1;
        X(2, 1) = xr2;
        X(1, 2) = xi1;
        X(2, 2) = xi2;
    }
    xnorm = std::max(std::fabs(xr1) + std::fabs(xi1), std::fabs(xr2) + std::fabs(xi2));
    if (xnorm > 1.0 && cmax > 1.0) {
        if (xnorm > bignum / cmax) {
            const double temp = cmax / bignum;
            X(1, 1) *= temp;
            X(2, 1) *= temp;
            X(1, 2) *= temp;
            X(2, 2) *= temp;
            xnorm *= temp;
            scale *= temp;
        }
    }
    return info;
#undef A
#undef B
#undef X
}

// ---------------------------------------------------------------- dtrevc ----
// Right eigenvectors of the upper quasi-triangular T (side = 'R').
// howmny: 'A' all (VR = eigenvectors of T), 'B' back-transformed by the input
// VR, 'S' selected (select[] standardised as LAPACK does).  work: 3n.
// Returns m (number of columns produced).
int trevc_right(char howmny, int* select, int n, const double* t, int ldt, double* vr, int ldvr,
                double* work) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
#define VR(i, j) vr[((i)-1) + (size_t)((j)-1) * ldvr]
#define WORK(i) work[(i)-1]
    const bool over = howmny == 'B', somev = howmny == 'S';
    int m = n;
    if (somev) {
        m = 0;
        bool pair = false;
        for (int j = 1; j <= n; ++j) {
            if (pair) {
                pair = false;
                select[j - 1] = 0;
            } else if (j < n) {
                if (T(j + 1, j) == 0.0) {
                    if (select[j - 1]) ++m;
                } else {
                    pair = true;
                    if (select[j - 1] || select[j]) {
                        select[j - 1] = 1;
                        m += 2;
                    }
                }
            } else if (select[n - 1]) {
                ++m;
            }
        }
    }
    if (n == 0) return m;
    const double unfl = kSafmin;
    const double ulp = kUlp;
    const double smlnum = unfl * (n / ulp);
    const double bignum = (1.0 - ulp) / smlnum;
    WORK(1) = 0.0;
    for (int j = 2; j <= n; ++j) {
        WORK(j) = 0.0;
        for (int i = 1; i <= j - 1; ++i) WORK(j) += std::fabs(T(i, j));
    }
    const int n2 = 2 * n;
    double x[4];  // X(2,2), ldx = 2
    auto daxpy = [&](int len, double alpha, const double* xs, double* ys) { axpy(len, alpha, xs, ys); };
    auto dscal = [&](int len, double alpha, double* xs) {
        for (int q = 0; q < len; ++q) xs[q] *= alpha;
    };
    auto idamax = [&](int len, const double* xs) {
        int best = 0;
        double bv = std::fabs(xs[0]);
        for (int q = 1; q < len; ++q)
            if (std::fabs(xs[q]) > bv) {
                bv = std::fabs(xs[q]);
                best = q;
            }
        return best;
    };
    // y = A(n x k) * xv + beta * y  (dgemv 'N')
    auto dgemv_n = [&](int k, const double* xv, double beta, double* y) {
        for (int r = 0; r < n; ++r) y[r] *= beta;
        for (int c = 0; c < k; ++c) {
            const double tmp = xv[c];
            if (tmp != 0.0)
                for (int r = 0; r < n; ++r) y[r] += tmp * vr[r + (size_t)c * ldvr];
        }
    };
    int ip = 0;
    int is = m;
    for (int ki = n; ki >= 1; --ki) {
        if (ip == 1) goto next;
        if (ki != 1 && T(ki, ki - 1) != 0.0) ip = -1;
        if (somev) {
            if (ip == 0) {
                if (!select[ki - 1]) goto next;
            } else {
                if (!select[ki - 2]) goto next;
            }
        }
        {
            const double wr = T(ki, ki);
            double wi = 0.0;
            if (ip != 0) wi = std::sqrt(std::fabs(T(ki, ki - 1))) * std::sqrt(std::fabs(T(ki - 1, ki)));
            const double smin = std::max(ulp * (std::fabs(wr) + std::fabs(wi)), smlnum);
            if (ip == 0) {
                WORK(ki + n) = 1.0;
                for (int k = 1; k <= ki - 1; ++k) WORK(k + n) = -T(k, ki);
                int jnxt = ki - 1;
                for (int j = ki - 1; j >= 1; --j) {
                    if (j > jnxt) continue;
                    int j1 = j, j2 = j;
                    jnxt = j - 1;
                    if (j > 1 && T(j, j - 1) != 0.0) {
                        j1 = j - 1;
                        jnxt = j - 2;
                    }
                    double scale, xnorm;
                    if (j1 == j2) {
                        laln2(1, 1, smin, 1.0, &T(j, j), ldt, 1.0, 1.0, &WORK(j + n), n, wr, 0.0, x, 2,
                              scale, xnorm);
                        if (xnorm > 1.0 && WORK(j) > bignum / xnorm) {
                            x[0] /= xnorm;
                            scale /= xnorm;
                        }
                        if (scale != 1.0) dscal(ki, scale, &WORK(1 + n));
                        WORK(j + n) = x[0];
                        daxpy(j - 1, -x[0], &T(1, j), &WORK(1 + n));
                    } else {
                        laln2(2, 1, smin, 1.0, &T(j - 1, j - 1), ldt, 1.0, 1.0, &WORK(j - 1 + n), n, wr,
                              0.0, x, 2, scale, xnorm);
                        if (xnorm > 1.0) {
                            const double beta = std::max(WORK(j - 1), WORK(j));
                            if (beta > bignum / xnorm) {
                                x[0] /= xnorm;
                                x[1] /= xnorm;
                                scale /= xnorm;
                            }
                        }
                        if (scale != 1.0) dscal(ki, scale, &WORK(1 + n));
                        WORK(j - 1 + n) = x[0];
                        WORK(j + n) = x[1];
                        daxpy(j - 2, -x[0], &T(1, j - 1), &WORK(1 + n));
                        daxpy(j - 2, -x[1], &T(1, j), &WORK(1 + n));
                    }
                }
                if (!over) {
                    std::memcpy(&VR(1, is), &WORK(1 + n), sizeof(double) * ki);
                    const int ii = idamax(ki, &VR(1, is));
                    const double remax = 1.0 / std::fabs(VR(ii + 1, is));
                    dscal(ki, remax, &VR(1, is));
                    for (int k = ki + 1; k <= n; ++k) VR(k, is) = 0.0;
                } else {
                    if (ki > 1) dgemv_n(ki - 1, &WORK(1 + n), WORK(ki + n), &VR(1, ki));
                    const int ii = idamax(n, &VR(1, ki));
                    const double remax = 1.0 / std::fabs(VR(ii + 1, ki));
                    dscal(n, remax, &VR(1, ki));
                }
            } else {
                if (std::fabs(T(ki - 1, ki)) >= std::fabs(T(ki, ki - 1))) {
                    WORK(ki - 1 + n) = 1.0;
                    WORK(ki + n2) = wi / T(ki - 1, ki);
                } else {
                    WORK(ki - 1 + n) = -wi / T(ki, ki - 1);
                    WORK(ki + n2) = 1.0;
                }
                WORK(ki + n) = 0.0;
                WORK(ki - 1 + n2) = 0.0;
                for (int k = 1; k <= ki - 2; ++k) {
                    WORK(k + n) = -WORK(ki - 1 + n) * T(k, ki - 1);
                    WORK(k + n2) = -WORK(ki + n2) * T(k, ki);
                }
                int jnxt = ki - 2;
                for (int j = ki - 2; j >= 1; --j) {
                    if (j > jnxt) continue;
                    int j1 = j, j2 = j;
                    jnxt = j - 1;
                    if (j > 1 && T(j, j - 1) != 0.0) {
                        j1 = j - 1;
                        jnxt = j - 2;
                    }
                    double scale, xnorm;
                    if (j1 == j2) {
                        laln2(1, 2, smin, 1.0, &T(j, j), ldt, 1.0, 1.0, &WORK(j + n), n, wr, wi, x, 2,
                              scale, xnorm);
                        if (xnorm > 1.0 && WORK(j) > bignum / xnorm) {
                            x[0] /= xnorm;
                            x[2] /= xnorm;
                            scale /= xnorm;
                        }
                        if (scale != 1.0) {
                            dscal(ki, scale, &WORK(1 + n));
                            dscal(ki, scale, &WORK(1 + n2));
                        }
                        WORK(j + n) = x[0];
                        WORK(j + n2) = x[2];
                        daxpy(j - 1, -x[0], &T(1, j), &WORK(1 + n));
                        daxpy(j - 1, -x[2], &T(1, j), &WORK(1 + n2));
                    } else {
                        laln2(2, 2, smin, 1.0, &T(j - 1, j - 1), ldt, 1.0, 1.0, &WORK(j - 1 + n), n, wr,
                              wi, x, 2, scale, xnorm);
                        if (xnorm > 1.0) {
                            const double beta = std::max(WORK(j - 1), WORK(j));
                            if (beta > bignum / xnorm) {
                                const double rec = 1.0 / xnorm;
                                x[0] *= rec;
                                x[2] *= rec;
                                x[1] *= rec;
                                x[3] *= rec;
                                scale *= rec;
                            }
                        }
                        if (scale != 1.0) {
                            dscal(ki, scale, &WORK(1 + n));
                            dscal(ki, scale, &WORK(1 + n2));
                        }
                        WORK(j - 1 + n) = x[0];
                        WORK(j + n) = x[1];
                        WORK(j - 1 + n2) = x[2];
                        WORK(j + n2) = x[3];
                        daxpy(j - 2, -x[0], &T(1, j - 1), &WORK(1 + n));
                        daxpy(j - 2, -x[1], &T(1, j), &WORK(1 + n));
                        daxpy(j - 2, -x[2], &T(1, j - 1), &WORK(1 + n2));
                        daxpy(j - 2, -x[3], &T(1, j), &WORK(1 + n2));
                    }
                }
                if (!over) {
                    std::memcpy(&VR(1, is - 1), &WORK(1 + n), sizeof(double) * ki);
                    std::memcpy(&VR(1, is), &WORK(1 + n2), sizeof(double) * ki);
                    double emax = 0.0;
                    for (int k = 1; k <= ki; ++k)
                        emax = std::max(emax, std::fabs(VR(k, is - 1)) + std::fabs(VR(k, is)));
                    const double remax = 1.0 / emax;
                    dscal(ki, remax, &VR(1, is - 1));
                    dscal(ki, remax, &VR(1, is));
                    for (int k = ki + 1; k <= n; ++k) {
                        VR(k, is - 1) = 0.0;
                        VR(k, is) = 0.0;
                    }
                } else {
                    if (ki > 2) {
                        dgemv_n(ki - 2, &WORK(1 + n), WORK(ki - 1 + n), &VR(1, ki - 1));
                        dgemv_n(ki - 2, &WORK(1 + n2), WORK(ki + n2), &VR(1, ki));
                    } else {
                        dscal(n, WORK(ki - 1 + n), &VR(1, ki - 1));
                        dscal(n, WORK(ki + n2), &VR(1, ki));
                    }
                    double emax = 0.0;
                    for (int k = 1; k <= n; ++k)
                        emax = std::max(emax, std::fabs(VR(k, ki - 1)) + std::fabs(VR(k, ki)));
                    const double remax = 1.0 / emax;
                    dscal(n, remax, &VR(1, ki - 1));
                    dscal(n, remax, &VR(1, ki));
                }
            }
            --is;
            if (ip != 0) --is;
        }
    next:
        if (ip == 1) ip = 0;
        if (ip == -1) ip = 1;
    }
    return m;
#undef T
#undef VR
#undef WORK
}

// ------------------------------------------------------ ARPACK nonsymmetric --
// dsortc (SRC/dsortc.f): shell sort of (xr, xi) by `which`, permuting y.
void dsortc(Which which, bool apply, int n, double* xr, double* xi, double* y) {
    auto ooo = [&](int a, int b) -> bool {
        switch (which) {
            case Which::LM: return lapy2(xr[a], xi[a]) > lapy2(xr[b], xi[b]);
            case Which::SM: return lapy2(xr[a], xi[a]) < lapy2(xr[b], xi[b]);
            case Which::LR: return xr[a] > xr[b];
            case Which::SR: return xr[a] < xr[b];
            case Which::LI: return std::fabs(xi[a]) > std::fabs(xi[b]);
            case Which::SI: return std::fabs(xi[a]) < std::fabs(xi[b]);
            default: return false;
        }
    };
    for (int igap = n / 2; igap != 0; igap /= 2) {
        for (int i = igap; i <= n - 1; ++i) {
            for (int j = i - igap; j >= 0; j -= igap) {
                if (!ooo(j, j + igap)) break;
                std::swap(xr[j], xr[j + igap]);
                std::swap(xi[j], xi[j + igap]);
                if (apply) std::swap(y[j], y[j + igap]);
            }
        }
    }
}

// dngets (SRC/dngets.f): sort so the wanted Ritz values are last; keep complex
// pairs together across the np | kev boundary; sort shifts by bounds.
void dngets(int ishift, Which which, int& kev, int& np, double* ritzr, double* ritzi,
            double* bounds) {
    const int n = kev + np;
    switch (which) {
        case Which::LM: dsortc(Which::LR, true, n, ritzr, ritzi, bounds); break;
        case Which::SM: dsortc(Which::SR, true, n, ritzr, ritzi, bounds); break;
        case Which::LR: dsortc(Which::LM, true, n, ritzr, ritzi, bounds); break;
        case Which::SR: dsortc(Which::SM, true, n, ritzr, ritzi, bounds); break;
        case Which::LI: dsortc(Which::LM, true, n, ritzr, ritzi, bounds); break;
        case Which::SI: dsortc(Which::SM, true, n, ritzr, ritzi, bounds); break;
        default: break;
    }
    dsortc(which, true, n, ritzr, ritzi, bounds);
    if ((ritzr[np] - ritzr[np - 1]) == 0.0 && (ritzi[np] + ritzi[np - 1]) == 0.0) {
        np -= 1;
        kev += 1;
    }
    if (ishift == 1) dsortc(Which::SR, true, np, bounds, ritzr, ritzi);
}

// dnconv (SRC/dnconv.f)
int dnconv(int n, const double* ritzr, const double* ritzi, const double* bounds, double tol,
           double eps) {
    const double eps23 = std::pow(eps, 2.0 / 3.0);
    int nconv = 0;
    for (int i = 0; i < n; ++i) {
        const double temp = std::max(eps23, lapy2(ritzr[i], ritzi[i]));
        if (bounds[i] <= tol * temp) ++nconv;
    }
    return nconv;
}

// dneigh (SRC/dneigh.f): Ritz values of H and their error bounds.
// workl >= n*n + 3n; q(ldq, n) receives the eigenvectors of the Schur form.
int dneigh(double rnorm, int n, const double* h, int ldh, double* ritzr, double* ritzi,
           double* bounds, double* q, int ldq, double* workl) {
    for (int j = 0; j < n; ++j) std::memcpy(workl + (size_t)j * n, h + (size_t)j * ldh, sizeof(double) * n);
    for (int j = 0; j < n - 1; ++j) bounds[j] = 0.0;
    bounds[n - 1] = 1.0;
    int ierr = lahqr(true, true, n, 1, n, workl, n, ritzr, ritzi, 1, 1, bounds, 1);
    if (ierr != 0) return ierr;
    std::vector<int> sel(n, 0);
    trevc_right('A', sel.data(), n, workl, n, q, ldq, workl + (size_t)n * n);
    int iconj = 0;
    for (int i = 0; i < n; ++i) {
        double* qi = q + (size_t)i * ldq;
        if (std::fabs(ritzi[i]) <= 0.0) {
            const double temp = nrm2(n, qi, 1);
            const double s = 1.0 / temp;
            for (int r = 0; r < n; ++r) qi[r] *= s;
        } else if (iconj == 0) {
            const double temp = lapy2(nrm2(n, qi, 1), nrm2(n, qi + ldq, 1));
            const double s = 1.0 / temp;
            for (int r = 0; r < n; ++r) qi[r] *= s;
            for (int r = 0; r < n; ++r) qi[ldq + r] *= s;
            iconj = 1;
        } else {
            iconj = 0;
        }
    }
    // workl(1:n) = Q' * bounds  (dgemv 'T')
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int r = 0; r < n; ++r) s += q[r + (size_t)i * ldq] * bounds[r];
        workl[i] = s;
    }
    iconj = 0;
    for (int i = 0; i < n; ++i) {
        if (std::fabs(ritzi[i]) <= 0.0) {
            bounds[i] = rnorm * std::fabs(workl[i]);
        } else if (iconj == 0) {
            bounds[i] = rnorm * lapy2(workl[i], workl[i + 1]);
            bounds[i + 1] = bounds[i];
            iconj = 1;
        } else {
            iconj = 0;
        }
    }
    return 0;
}

// Bulge chase of dnapps (SRC/dnapps.f:236-545) on the host: applies the np
// shifts to H (ldh) and accumulates Q (ldq x kplusp).  nglob is the problem
// dimension (it enters smlnum).  Returns the (possibly incremented) kev; the
// n-length V*Q / residual update is done on the device by the caller.
int dnapps_host(int kev, int np, const double* shiftr, const double* shifti, double* h, int ldh,
                double* q, int ldq, double* workl, int64_t nglob) {
#define H(i, j) h[((i)-1) + (size_t)((j)-1) * ldh]
#define Q(i, j) q[((i)-1) + (size_t)((j)-1) * ldq]
    const double unfl = kSafmin;
    const double ulp = kUlp;
    const double smlnum = unfl * ((double)nglob / ulp);
    const int kplusp = kev + np;
    for (int j = 1; j <= kplusp; ++j)
        for (int i = 1; i <= kplusp; ++i) Q(i, j) = (i == j) ? 1.0 : 0.0;
    if (np == 0) return kev;
    bool cconj = false;
    for (int jj = 1; jj <= np; ++jj) {
        const double sigmar = shiftr[jj - 1], sigmai = shifti[jj - 1];
        if (cconj) {
            cconj = false;
            continue;
        } else if (jj < np && std::fabs(sigmai) > 0.0) {
            cconj = true;
        } else if (jj == np && std::fabs(sigmai) > 0.0) {
            kev = kev + 1;
            continue;
        }
        int istart = 1;
        for (;;) {  // label 20
            int iend = kplusp;
            for (int i = istart; i <= kplusp - 1; ++i) {
                double tst1 = std::fabs(H(i, i)) + std::fabs(H(i + 1, i + 1));
                if (tst1 == 0.0) tst1 = lanhs1(kplusp - jj + 1, h, ldh);
                if (std::fabs(H(i + 1, i)) <= std::max(ulp * tst1, smlnum)) {
                    iend = i;
                    H(i + 1, i) = 0.0;
                    break;
                }
            }
            if (istart == iend || (istart + 1 == iend && std::fabs(sigmai) > 0.0)) {
                // nothing to chase in this block
            } else {
                const double h11 = H(istart, istart), h21 = H(istart + 1, istart);
                if (std::fabs(sigmai) <= 0.0) {  // real shift: Givens bulge chase
                    double f = h11 - sigmar, g = h21;
                    for (int i = istart; i <= iend - 1; ++i) {
                        double c, s, r;
                        lartg(f, g, c, s, r);
                        if (i > istart) {
                            if (r < 0.0) {
                                r = -r;
                                c = -c;
                                s = -s;
                            }
                            H(i, i - 1) = r;
                            H(i + 1, i - 1) = 0.0;
                        }
                        for (int j = i; j <= kplusp; ++j) {
                            const double t = c * H(i, j) + s * H(i + 1, j);
                            H(i + 1, j) = -s * H(i, j) + c * H(i + 1, j);
                            H(i, j) = t;
                        }
                        for (int j = 1; j <= std::min(i + 2, iend); ++j) {
                            const double t = c * H(j, i) + s * H(j, i + 1);
                            H(j, i + 1) = -s * H(j, i) + c * H(j, i + 1);
                            H(j, i) = t;
                        }
                        for (int j = 1; j <= std::min(i + jj, kplusp); ++j) {
                            const double t = c * Q(j, i) + s * Q(j, i + 1);
                            Q(j, i + 1) = -s * Q(j, i) + c * Q(j, i + 1);
                            Q(j, i) = t;
                        }
                        if (i < iend - 1) {
                            f = H(i + 1, i);
                            g = H(i + 2, i);
                        }
                    }
                } else {  // complex conjugate pair: double-shift Householder chase
                    const double h12 = H(istart, istart + 1), h22 = H(istart + 1, istart + 1);
                    const double h32 = H(istart + 2, istart + 1);
                    const double s = 2.0 * sigmar;
                    const double t = lapy2(sigmar, sigmai);
                    double u[3];
                    u[0] = (h11 * (h11 - s) + t * t) / h21 + h12;
                    u[1] = h11 + h22 - s;
                    u[2] = h32;
                    for (int i = istart; i <= iend - 1; ++i) {
                        const int nr = std::min(3, iend - i + 1);
                        double tau;
                        larfg(nr, u[0], u + 1, 1, tau);
                        if (i > istart) {
                            H(i, i - 1) = u[0];
                            H(i + 1, i - 1) = 0.0;
                            if (i < iend - 1) H(i + 2, i - 1) = 0.0;
                        }
                        u[0] = 1.0;
                        larf('L', nr, kplusp - i + 1, u, 1, tau, &H(i, i), ldh, workl);
                        const int ir = std::min(i + 3, iend);
                        larf('R', ir, nr, u, 1, tau, &H(1, i), ldh, workl);
                        larf('R', kplusp, nr, u, 1, tau, &Q(1, i), ldq, workl);
                        if (i < iend - 1) {
                            u[0] = H(i + 1, i);
                            u[1] = H(i + 2, i);
                            if (i < iend - 2) u[2] = H(i + 3, i);
                        }
                    }
                }
            }
            istart = iend + 1;
            if (iend >= kplusp) break;
        }
    }
    // make the subdiagonals of the kev block non-negative (SRC/dnapps.f:549-555)
    for (int j = 1; j <= kev; ++j) {
        if (H(j + 1, j) < 0.0) {
            for (int c = j; c <= kplusp; ++c) H(j + 1, c) = -H(j + 1, c);  // dscal(kplusp-j+1, h(j+1,j), ldh)
            for (int r = 1; r <= std::min(j + 2, kplusp); ++r) H(r, j + 1) = -H(r, j + 1);
            for (int r = 1; r <= std::min(j + np + 1, kplusp); ++r) Q(r, j + 1) = -Q(r, j + 1);
        }
    }
    for (int i = 1; i <= kev; ++i) {  // final deflation check (SRC/dnapps.f:557-575)
        double tst1 = std::fabs(H(i, i)) + std::fabs(H(i + 1, i + 1));
        if (tst1 == 0.0) tst1 = lanhs1(kev, h, ldh);
        if (H(i + 1, i) <= std::max(ulp * tst1, smlnum)) H(i + 1, i) = 0.0;
    }
    return kev;
#undef H
#undef Q
}

// ------------------------------------------------- Schur reordering (dneupd) --
namespace {
// dlarfx for an order-3 reflector (LAPACK's unrolled special case, scalar).
void larfx3(char side, int m, int n, const double* v, double tau, double* c, int ldc) {
    if (tau == 0.0) return;
    const double v1 = v[0], v2 = v[1], v3 = v[2];
    const double t1 = tau * v1, t2 = tau * v2, t3 = tau * v3;
    if (side == 'L') {  // order m = 3
        for (int j = 0; j < n; ++j) {
            double* cj = c + (size_t)j * ldc;
            const double sum = v1 * cj[0] + v2 * cj[1] + v3 * cj[2];
            cj[0] -= sum * t1;
            cj[1] -= sum * t2;
            cj[2] -= sum * t3;
        }
    } else {  // order n = 3
        for (int j = 0; j < m; ++j) {
            double* c1 = c + j;
            const double sum = v1 * c1[0] + v2 * c1[ldc] + v3 * c1[2 * (size_t)ldc];
            c1[0] -= sum * t1;
            c1[ldc] -= sum * t2;
            c1[2 * (size_t)ldc] -= sum * t3;
        }
    }
}
// drot over n pairs (x, y) with strides (OpenBLAS arithmetic, see rot_x/rot_y)
void drot(int n, double* x, int incx, double* y, int incy, double c, double s) {
    for (int i = 0; i < n; ++i) {
        const double a = x[(size_t)i * incx], b = y[(size_t)i * incy];
        x[(size_t)i * incx] = rot_x(c, s, a, b);
        y[(size_t)i * incy] = rot_y(c, s, a, b);
    }
}
}  // namespace

// dlasy2 (ltranl = ltranr = false): TL*X + isgn*X*TR = scale*B, n1,n2 in {1,2}.
int lasy2(int isgn, int n1, int n2, const double* tl, int ldtl, const double* tr, int ldtr,
          const double* b, int ldb, double& scale, double* x, int ldx, double& xnorm) {
#define TL(i, j) tl[((i)-1) + (size_t)((j)-1) * ldtl]
#define TR(i, j) tr[((i)-1) + (size_t)((j)-1) * ldtr]
#define B(i, j) b[((i)-1) + (size_t)((j)-1) * ldb]
#define X(i, j) x[((i)-1) + (size_t)((j)-1) * ldx]
    static const int locu12[4] = {3, 4, 1, 2}, locl21[4] = {2, 1, 4, 3}, locu22[4] = {4, 3, 2, 1};
    static const bool xswpiv[4] = {false, false, true, true}, bswpiv[4] = {false, true, false, true};
    int info = 0;
    if (n1 == 0 || n2 == 0) return 0;
    const double eps = kUlp;
    const double smlnum = kSafmin / eps;
    const double sgn = isgn;
    const int k = n1 + n1 + n2 - 2;
    double tmp[4], btmp[4], x2[2];
    if (k == 1) {
        double tau1 = TL(1, 1) + sgn * TR(1, 1);
        double bet = std::fabs(tau1);
        if (bet <= smlnum) {
            tau1 = smlnum;
            bet = smlnum;
            info = 1;
        }
        scale = 1.0;
        const double gam = std::fabs(B(1, 1));
        if (smlnum * gam > bet) scale = 1.0 / gam;
        X(1, 1) = (B(1, 1) * scale) / tau1;
        xnorm = std::fabs(X(1, 1));
        return info;
    }
    if (k == 2 || k == 3) {
        double smin;
        if (k == 2) {  // 1 x 2
            smin = std::max(eps * std::max({std::fabs(TL(1, 1)), std::fabs(TR(1, 1)), std::fabs(TR(1, 2)),
                                            std::fabs(TR(2, 1)), std::fabs(TR(2, 2))}),
                            smlnum);
            tmp[0] = TL(1, 1) + sgn * TR(1, 1);
            tmp[3] = TL(1, 1) + sgn * TR(2, 2);
            tmp[1] = sgn * TR(1, 2);
            tmp[2] = sgn * TR(2, 1);
            btmp[0] = B(1, 1);
            btmp[1] = B(1, 2);
        } else {  // 2 x 1
            smin = std::max(eps * std::max({std::fabs(TR(1, 1)), std::fabs(TL(1, 1)), std::fabs(TL(1, 2)),
                                            std::fabs(TL(2, 1)), std::fabs(TL(2, 2))}),
                            smlnum);
            tmp[0] = TL(1, 1) + sgn * TR(1, 1);
            tmp[3] = TL(2, 2) + sgn * TR(1, 1);
            tmp[1] = TL(2, 1);
            tmp[2] = TL(1, 2);
            btmp[0] = B(1, 1);
            btmp[1] = B(2, 1);
        }
        int ipiv = 0;
        for (int q = 1; q < 4; ++q)
            if (std::fabs(tmp[q]) > std::fabs(tmp[ipiv])) ipiv = q;
        double u11 = tmp[ipiv];
        if (std::fabs(u11) <= smin) {
            info = 1;
            u11 = smin;
        }
        const double u12 = tmp[locu12[ipiv] - 1];
        const double l21 = tmp[locl21[ipiv] - 1] / u11;
        double u22 = tmp[locu22[ipiv] - 1] - u12 * l21;
        const bool xswap = xswpiv[ipiv], bswap = bswpiv[ipiv];
        if (std::fabs(u22) <= smin) {
            info = 1;
            u22 = smin;
        }
        if (bswap) {
            const double temp = btmp[1];
            btmp[1] = btmp[0] - l21 * temp;
            btmp[0] = temp;
        } else {
            btmp[1] = btmp[1] - l21 * btmp[0];
        }
        scale = 1.0;
        if ((2.0 * smlnum) * std::fabs(btmp[1]) > std::fabs(u22) ||
            (2.0 * smlnum) * std::fabs(btmp[0]) > std::fabs(u11)) {
            scale = 0.5 / std::max(std::fabs(btmp[0]), std::fabs(btmp[1]));
            btmp[0] *= scale;
            btmp[1] *= scale;
        }
        x2[1] = btmp[1] / u22;
        x2[0] = btmp[0] / u11 - (u12 / u11) * x2[1];
        if (xswap) std::swap(x2[0], x2[1]);
        X(1, 1) = x2[0];
        if (n1 == 1) {
            X(1, 2) = x2[1];
            xnorm = std::fabs(X(1, 1)) + std::fabs(X(1, 2));
        } else {
            X(2, 1) = x2[1];
            xnorm = std::max(std::fabs(X(1, 1)), std::fabs(X(2, 1)));
        }
        return info;
    }
    // 2 x 2: equivalent 4 x 4 system, complete pivoting
    double smin = std::max({std::fabs(TR(1, 1)), std::fabs(TR(1, 2)), std::fabs(TR(2, 1)), std::fabs(TR(2, 2))});
    smin = std::max({smin, std::fabs(TL(1, 1)), std::fabs(TL(1, 2)), std::fabs(TL(2, 1)), std::fabs(TL(2, 2))});
    smin = std::max(eps * smin, smlnum);
    double t16[4][4] = {};  // t16[col][row] (column-major like the reference)
#define T16(i, j) t16[(j)-1][(i)-1]
    T16(1, 1) = TL(1, 1) + sgn * TR(1, 1);
    T16(2, 2) = TL(2, 2) + sgn * TR(1, 1);
    T16(3, 3) = TL(1, 1) + sgn * TR(2, 2);
    T16(4, 4) = TL(2, 2) + sgn * TR(2, 2);
    T16(1, 2) = TL(1, 2);
    T16(2, 1) = TL(2, 1);
    T16(3, 4) = TL(1, 2);
    T16(4, 3) = TL(2, 1);
    T16(1, 3) = sgn * TR(2, 1);
    T16(2, 4) = sgn * TR(2, 1);
    T16(3, 1) = sgn * TR(1, 2);
    T16(4, 2) = sgn * TR(1, 2);
    btmp[0] = B(1, 1);
    btmp[1] = B(2, 1);
    btmp[2] = B(1, 2);
    btmp[3] = B(2, 2);
    int jpiv[4] = {0, 0, 0, 0};
    for (int i = 1; i <= 3; ++i) {
        double xmax = 0.0;
        int ipsv = i, jpsv = i;
        for (int ip = i; ip <= 4; ++ip)
            for (int jp = i; jp <= 4; ++jp)
                if (std::fabs(T16(ip, jp)) >= xmax) {
                    xmax = std::fabs(T16(ip, jp));
                    ipsv = ip;
                    jpsv = jp;
                }
        if (ipsv != i) {
            for (int c = 1; c <= 4; ++c) std::swap(T16(ipsv, c), T16(i, c));
            std::swap(btmp[i - 1], btmp[ipsv - 1]);
        }
        if (jpsv != i)
            for (int r = 1; r <= 4; ++r) std::swap(T16(r, jpsv), T16(r, i));
        jpiv[i - 1] = jpsv;
        if (std::fabs(T16(i, i)) < smin) {
            info = 1;
            T16(i, i) = smin;
        }
        for (int j = i + 1; j <= 4; ++j) {
            T16(j, i) = T16(j, i) / T16(i, i);
            btmp[j - 1] = btmp[j - 1] - T16(j, i) * btmp[i - 1];
            for (int kk = i + 1; kk <= 4; ++kk) T16(j, kk) = T16(j, kk) - T16(j, i) * T16(i, kk);
        }
    }
    if (std::fabs(T16(4, 4)) < smin) {
        info = 1;
        T16(4, 4) = smin;
    }
    scale = 1.0;
    if ((8.0 * smlnum) * std::fabs(btmp[0]) > std::fabs(T16(1, 1)) ||
        (8.0 * smlnum) * std::fabs(btmp[1]) > std::fabs(T16(2, 2)) ||
        (8.0 * smlnum) * std::fabs(btmp[2]) > std::fabs(T16(3, 3)) ||
        (8.0 * smlnum) * std::fabs(btmp[3]) > std::fabs(T16(4, 4))) {
        scale = (1.0 / 8.0) / std::max({std::fabs(btmp[0]), std::fabs(btmp[1]), std::fabs(btmp[2]),
                                         std::fabs(btmp[3])});
        for (double& bb : btmp) bb *= scale;
    }
    for (int i = 1; i <= 4; ++i) {
        const int kk = 5 - i;
        const double temp = 1.0 / T16(kk, kk);
        tmp[kk - 1] = btmp[kk - 1] * temp;
        for (int j = kk + 1; j <= 4; ++j) tmp[kk - 1] = tmp[kk - 1] - (temp * T16(kk, j)) * tmp[j - 1];
    }
    for (int i = 1; i <= 3; ++i) {
        const int kk = 4 - i;
        if (jpiv[kk - 1] != kk) std::swap(tmp[kk - 1], tmp[jpiv[kk - 1] - 1]);
    }
    X(1, 1) = tmp[0];
    X(2, 1) = tmp[1];
    X(1, 2) = tmp[2];
    X(2, 2) = tmp[3];
    xnorm = std::max(std::fabs(tmp[0]) + std::fabs(tmp[2]), std::fabs(tmp[1]) + std::fabs(tmp[3]));
    return info;
#undef T16
#undef TL
#undef TR
#undef B
#undef X
}

// dlaexc: swap adjacent diagonal blocks T11 (n1) and T22 (n2) at row j1 (1-based).
int laexc(bool wantq, int n, double* t, int ldt, double* q, int ldq, int j1, int n1, int n2,
          double* work) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
#define Q(i, j) q[((i)-1) + (size_t)((j)-1) * ldq]
    (void)work;
    if (n == 0 || n1 == 0 || n2 == 0) return 0;
    if (j1 + n1 > n) return 0;
    const int j2 = j1 + 1, j3 = j1 + 2, j4 = j1 + 3;
    if (n1 == 1 && n2 == 1) {
        const double t11 = T(j1, j1), t22 = T(j2, j2);
        double cs, sn, temp;
        lartg(T(j1, j2), t22 - t11, cs, sn, temp);
        if (j3 <= n) drot(n - j1 - 1, &T(j1, j3), ldt, &T(j2, j3), ldt, cs, sn);
        drot(j1 - 1, &T(1, j1), 1, &T(1, j2), 1, cs, sn);
        T(j1, j1) = t22;
        T(j2, j2) = t11;
        if (wantq) drot(n, &Q(1, j1), 1, &Q(1, j2), 1, cs, sn);
        return 0;
    }
    const int nd = n1 + n2;
    double d[16];  // D(4,4), ldd = 4
#define D(i, j) d[((i)-1) + ((j)-1) * 4]
    double dnorm = 0.0;
    for (int j = 1; j <= nd; ++j)
        for (int i = 1; i <= nd; ++i) {
            D(i, j) = T(j1 + i - 1, j1 + j - 1);
            const double a = std::fabs(D(i, j));
            if (dnorm < a || std::isnan(a)) dnorm = a;
        }
    const double eps = kUlp;
    const double smlnum = kSafmin / eps;
    const double thresh = std::max(10.0 * eps * dnorm, smlnum);
    double x[4], scale, xnorm;  // X(2,2), ldx = 2
    lasy2(-1, n1, n2, d, 4, &D(n1 + 1, n1 + 1), 4, &D(1, n1 + 1), 4, scale, x, 2, xnorm);
    const int k = n1 + n1 + n2 - 3;
    if (k == 1) {  // n1 = 1, n2 = 2
        double u[3] = {scale, x[0], x[2]};
        double tau;
        larfg(3, u[2], u, 1, tau);
        u[2] = 1.0;
        const double t11 = T(j1, j1);
        larfx3('L', 3, 3, u, tau, d, 4);
        larfx3('R', 3, 3, u, tau, d, 4);
        if (std::max({std::fabs(D(3, 1)), std::fabs(D(3, 2)), std::fabs(D(3, 3) - t11)}) > thresh) return 1;
        larfx3('L', 3, n - j1 + 1, u, tau, &T(j1, j1), ldt);
        larfx3('R', j2, 3, u, tau, &T(1, j1), ldt);
        T(j3, j1) = 0.0;
        T(j3, j2) = 0.0;
        T(j3, j3) = t11;
        if (wantq) larfx3('R', n, 3, u, tau, &Q(1, j1), ldq);
    } else if (k == 2) {  // n1 = 2, n2 = 1
        double u[3] = {-x[0], -x[1], scale};
        double tau;
        larfg(3, u[0], u + 1, 1, tau);
        u[0] = 1.0;
        const double t33 = T(j3, j3);
        larfx3('L', 3, 3, u, tau, d, 4);
        larfx3('R', 3, 3, u, tau, d, 4);
        if (std::max({std::fabs(D(2, 1)), std::fabs(D(3, 1)), std::fabs(D(1, 1) - t33)}) > thresh) return 1;
        larfx3('R', j3, 3, u, tau, &T(1, j1), ldt);
        larfx3('L', 3, n - j1, u, tau, &T(j1, j2), ldt);
        T(j1, j1) = t33;
        T(j2, j1) = 0.0;
        T(j3, j1) = 0.0;
        if (wantq) larfx3('R', n, 3, u, tau, &Q(1, j1), ldq);
    } else {  // n1 = 2, n2 = 2
        double u1[3] = {-x[0], -x[1], scale};
        double tau1;
        larfg(3, u1[0], u1 + 1, 1, tau1);
        u1[0] = 1.0;
        const double temp = -tau1 * (x[2] + u1[1] * x[3]);
        double u2[3] = {-temp * u1[1] - x[3], -temp * u1[2], scale};
        double tau2;
        larfg(3, u2[0], u2 + 1, 1, tau2);
        u2[0] = 1.0;
        // order-3 reflectors on the 4 x 4 block D
        larfx3('L', 3, 4, u1, tau1, d, 4);
        larfx3('R', 4, 3, u1, tau1, d, 4);
        larfx3('L', 3, 4, u2, tau2, &D(2, 1), 4);
        larfx3('R', 4, 3, u2, tau2, &D(1, 2), 4);
        if (std::max({std::fabs(D(3, 1)), std::fabs(D(3, 2)), std::fabs(D(4, 1)), std::fabs(D(4, 2))}) > thresh)
            return 1;
        larfx3('L', 3, n - j1 + 1, u1, tau1, &T(j1, j1), ldt);
        larfx3('R', j4, 3, u1, tau1, &T(1, j1), ldt);
        larfx3('L', 3, n - j1 + 1, u2, tau2, &T(j2, j1), ldt);
        larfx3('R', j4, 3, u2, tau2, &T(1, j2), ldt);
        T(j3, j1) = 0.0;
        T(j3, j2) = 0.0;
        T(j4, j1) = 0.0;
        T(j4, j2) = 0.0;
        if (wantq) {
            larfx3('R', n, 3, u1, tau1, &Q(1, j1), ldq);
            larfx3('R', n, 3, u2, tau2, &Q(1, j2), ldq);
        }
    }
#undef D
    double wr1, wi1, wr2, wi2, cs, sn;
    if (n2 == 2) {  // standardise the new 2 x 2 block T11
        lanv2(T(j1, j1), T(j1, j2), T(j2, j1), T(j2, j2), wr1, wi1, wr2, wi2, cs, sn);
        drot(n - j1 - 1, &T(j1, j1 + 2), ldt, &T(j2, j1 + 2), ldt, cs, sn);
        drot(j1 - 1, &T(1, j1), 1, &T(1, j2), 1, cs, sn);
        if (wantq) drot(n, &Q(1, j1), 1, &Q(1, j2), 1, cs, sn);
    }
    if (n1 == 2) {  // standardise the new 2 x 2 block T22
        const int k3 = j1 + n2, k4 = k3 + 1;
        lanv2(T(k3, k3), T(k3, k4), T(k4, k3), T(k4, k4), wr1, wi1, wr2, wi2, cs, sn);
        if (k3 + 2 <= n) drot(n - k3 - 1, &T(k3, k3 + 2), ldt, &T(k4, k3 + 2), ldt, cs, sn);
        drot(k3 - 1, &T(1, k3), 1, &T(1, k4), 1, cs, sn);
        if (wantq) drot(n, &Q(1, k3), 1, &Q(1, k4), 1, cs, sn);
    }
    return 0;
#undef T
#undef Q
}

// dtrexc: move the block at ifst to ilst (1-based, in/out).
int trexc(bool wantq, int n, double* t, int ldt, double* q, int ldq, int& ifst, int& ilst,
          double* work) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
    if (n <= 1) return 0;
    if (ifst > 1 && T(ifst, ifst - 1) != 0.0) --ifst;
    int nbf = 1;
    if (ifst < n && T(ifst + 1, ifst) != 0.0) nbf = 2;
    if (ilst > 1 && T(ilst, ilst - 1) != 0.0) --ilst;
    int nbl = 1;
    if (ilst < n && T(ilst + 1, ilst) != 0.0) nbl = 2;
    if (ifst == ilst) return 0;
    int here, info = 0;
    if (ifst < ilst) {
        if (nbf == 2 && nbl == 1) --ilst;
        if (nbf == 1 && nbl == 2) ++ilst;
        here = ifst;
        do {
            if (nbf == 1 || nbf == 2) {
                int nbnext = 1;
                if (here + nbf + 1 <= n && T(here + nbf + 1, here + nbf) != 0.0) nbnext = 2;
                info = laexc(wantq, n, t, ldt, q, ldq, here, nbf, nbnext, work);
                if (info != 0) {
                    ilst = here;
                    return info;
                }
                here += nbnext;
                if (nbf == 2 && T(here + 1, here) == 0.0) nbf = 3;
            } else {
                int nbnext = 1;
                if (here + 3 <= n && T(here + 3, here + 2) != 0.0) nbnext = 2;
                info = laexc(wantq, n, t, ldt, q, ldq, here + 1, 1, nbnext, work);
                if (info != 0) {
                    ilst = here;
                    return info;
                }
                if (nbnext == 1) {
                    laexc(wantq, n, t, ldt, q, ldq, here, 1, nbnext, work);
                    ++here;
                } else {
                    if (T(here + 2, here + 1) == 0.0) nbnext = 1;
                    if (nbnext == 2) {
                        info = laexc(wantq, n, t, ldt, q, ldq, here, 1, nbnext, work);
                        if (info != 0) {
                            ilst = here;
                            return info;
                        }
                        here += 2;
                    } else {
                        laexc(wantq, n, t, ldt, q, ldq, here, 1, 1, work);
                        laexc(wantq, n, t, ldt, q, ldq, here + 1, 1, 1, work);
                        here += 2;
                    }
                }
            }
        } while (here < ilst);
    } else {
        here = ifst;
        do {
            if (nbf == 1 || nbf == 2) {
                int nbnext = 1;
                if (here >= 3 && T(here - 1, here - 2) != 0.0) nbnext = 2;
                info = laexc(wantq, n, t, ldt, q, ldq, here - nbnext, nbnext, nbf, work);
                if (info != 0) {
                    ilst = here;
                    return info;
                }
                here -= nbnext;
                if (nbf == 2 && T(here + 1, here) == 0.0) nbf = 3;
            } else {
                int nbnext = 1;
                if (here >= 3 && T(here - 1, here - 2) != 0.0) nbnext = 2;
                info = laexc(wantq, n, t, ldt, q, ldq, here - nbnext, nbnext, 1, work);
                if (info != 0) {
                    ilst = here;
                    return info;
                }
                if (nbnext == 1) {
                    laexc(wantq, n, t, ldt, q, ldq, here, nbnext, 1, work);
                    --here;
                } else {
                    if (T(here, here - 1) == 0.0) nbnext = 1;
                    if (nbnext == 2) {
                        info = laexc(wantq, n, t, ldt, q, ldq, here - 1, 2, 1, work);
                        if (info != 0) {
                            ilst = here;
                            return info;
                        }
                        here -= 2;
                    } else {
                        laexc(wantq, n, t, ldt, q, ldq, here, 1, 1, work);
                        laexc(wantq, n, t, ldt, q, ldq, here - 1, 1, 1, work);
                        here -= 2;
                    }
                }
            }
        } while (here > ilst);
    }
    ilst = here;
    return 0;
#undef T
}

// dtrsen(job = 'N', compq = 'V'): move the selected eigenvalues to the leading
// block; wr/wi recomputed from T; m = dimension of the selected subspace.
int trsen(const int* select, int n, double* t, int ldt, double* q, int ldq, double* wr,
          double* wi, int& m, double* work) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
    m = 0;
    bool pair = false;
    for (int k = 1; k <= n; ++k) {
        if (pair) {
            pair = false;
        } else if (k < n) {
            if (T(k + 1, k) == 0.0) {
                if (select[k - 1]) ++m;
            } else {
                pair = true;
                if (select[k - 1] || select[k]) m += 2;
            }
        } else if (select[n - 1]) {
            ++m;
        }
    }
    int info = 0;
    if (!(m == n || m == 0)) {
        int ks = 0;
        pair = false;
        for (int k = 1; k <= n; ++k) {
            if (pair) {
                pair = false;
                continue;
            }
            bool swap = select[k - 1] != 0;
            if (k < n && T(k + 1, k) != 0.0) {
                pair = true;
                swap = swap || select[k] != 0;
            }
            if (swap) {
                ++ks;
                int ierr = 0, kk = k;
                if (k != ks) ierr = trexc(true, n, t, ldt, q, ldq, kk, ks, work);  // ks in/out
                if (ierr == 1 || ierr == 2) {
                    info = 1;
                    break;
                }
                if (pair) ++ks;
            }
        }
    }
    for (int k = 1; k <= n; ++k) {
        wr[k - 1] = T(k, k);
        wi[k - 1] = 0.0;
    }
    for (int k = 1; k <= n - 1; ++k)
        if (T(k + 1, k) != 0.0) {
            wi[k - 1] = std::sqrt(std::fabs(T(k, k + 1))) * std::sqrt(std::fabs(T(k + 1, k)));
            wi[k] = -wi[k - 1];
        }
    return info;
#undef T
}

}  // namespace ahip::la
