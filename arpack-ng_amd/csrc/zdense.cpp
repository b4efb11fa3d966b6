// Complex host kit (see zdense.hpp).  Complex division follows Fortran's
// range-reduced (Smith) rule that gfortran/flang compile the reference with.
#include "zdense.hpp"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

namespace ahip::zla {

namespace {
constexpr double kUlp = DBL_EPSILON;  // dlamch('P')
constexpr double kSafmin = DBL_MIN;

inline cd cdiv(cd x, cd y) {  // Smith's algorithm
    const double a = x.real(), b = x.imag(), c = y.real(), d = y.imag();
    if (std::fabs(c) < std::fabs(d)) {
        const double ratio = c / d, denom = c * ratio + d;
        return cd((a * ratio + b) / denom, (b * ratio - a) / denom);
    }
    const double ratio = d / c, denom = d * ratio + c;
    return cd((b * ratio + a) / denom, (b - a * ratio) / denom);
}
inline double abssq(cd t) { return t.real() * t.real() + t.imag() * t.imag(); }
inline double dlapy3(double x, double y, double z) {
    const double xa = std::fabs(x), ya = std::fabs(y), za = std::fabs(z);
    const double w = std::max({xa, ya, za});
    if (w == 0.0) return xa + ya + za;
    return w * std::sqrt((xa / w) * (xa / w) + (ya / w) * (ya / w) + (za / w) * (za / w));
}
// zrot: cx' = c*cx + s*cy ; cy' = c*cy - conj(s)*cx
inline void zrot(int n, cd* x, int incx, cd* y, int incy, double c, cd s) {
    for (int i = 0; i < n; ++i) {
        cd& a = x[(size_t)i * incx];
        cd& b = y[(size_t)i * incy];
        const cd t = c * a + s * b;
        b = c * b - std::conj(s) * a;
        a = t;
    }
}
}  // namespace

double dznrm2(int n, const cd* x, int incx) {
    if (n < 1) return 0.0;
    long double s = 0.0L;
    for (int i = 0; i < n; ++i) {
        const long double re = x[(size_t)i * incx].real(), im = x[(size_t)i * incx].imag();
        s += re * re + im * im;
    }
    return (double)std::sqrt(s);
}

double lanhs1(int n, const cd* a, int lda) {
    double value = 0.0;
    for (int j = 0; j < n; ++j) {
        double sum = 0.0;
        for (int i = 0; i <= std::min(n - 1, j + 1); ++i) sum += std::abs(a[i + (size_t)j * lda]);
        if (value < sum || std::isnan(sum)) value = sum;
    }
    return value;
}

void lartg(cd f, cd g, double& c, cd& s, cd& r) {
    const double safmin = kSafmin, safmax = 1.0 / kSafmin;
    const double rtmin = std::sqrt(safmin);
    if (g == cd(0.0)) {
        c = 1.0;
        s = 0.0;
        r = f;
    } else if (f == cd(0.0)) {
        c = 0.0;
        if (g.real() == 0.0) {
            r = std::fabs(g.imag());
            s = std::conj(g) / r.real();
        } else if (g.imag() == 0.0) {
            r = std::fabs(g.real());
            s = std::conj(g) / r.real();
        } else {
            const double g1 = std::max(std::fabs(g.real()), std::fabs(g.imag()));
            const double rtmax = std::sqrt(safmax / 2);
            if (g1 > rtmin && g1 < rtmax) {
                const double d = std::sqrt(abssq(g));
                s = std::conj(g) / d;
                r = d;
            } else {
                const double u = std::min(safmax, std::max(safmin, g1));
                const cd gs = g / u;
                const double d = std::sqrt(abssq(gs));
                s = std::conj(gs) / d;
                r = d * u;
            }
        }
    } else {
        const double f1 = std::max(std::fabs(f.real()), std::fabs(f.imag()));
        const double g1 = std::max(std::fabs(g.real()), std::fabs(g.imag()));
        double rtmax = std::sqrt(safmax / 4);
        if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
            const double f2 = abssq(f), g2 = abssq(g), h2 = f2 + g2;
            if (f2 >= h2 * safmin) {
                c = std::sqrt(f2 / h2);
                r = f / c;
                rtmax *= 2;
                if (f2 > rtmin && h2 < rtmax) s = std::conj(g) * (f / std::sqrt(f2 * h2));
                else s = std::conj(g) * (r / h2);
            } else {
                const double d = std::sqrt(f2 * h2);
                c = f2 / d;
                r = (c >= safmin) ? f / c : f * (h2 / d);
                s = std::conj(g) * (f / d);
            }
        } else {
            const double u = std::min(safmax, std::max({safmin, f1, g1}));
            const cd gs = g / u;
            const double g2 = abssq(gs);
            double w, f2, h2;
            cd fs;
            if (f1 / u < rtmin) {
                const double v = std::min(safmax, std::max(safmin, f1));
                w = v / u;
                fs = f / v;
                f2 = abssq(fs);
                h2 = f2 * w * w + g2;
            } else {
                w = 1.0;
                fs = f / u;
                f2 = abssq(fs);
                h2 = f2 + g2;
            }
            if (f2 >= h2 * safmin) {
                c = std::sqrt(f2 / h2);
                r = fs / c;
                rtmax *= 2;
                if (f2 > rtmin && h2 < rtmax) s = std::conj(gs) * (fs / std::sqrt(f2 * h2));
                else s = std::conj(gs) * (r / h2);
            } else {
                const double d = std::sqrt(f2 * h2);
                c = f2 / d;
                r = (c >= safmin) ? fs / c : fs * (h2 / d);
                s = std::conj(gs) * (fs / d);
            }
            c *= w;
            r *= u;
        }
    }
}

void larfg(int n, cd& alpha, cd* x, int incx, cd& tau) {
    if (n <= 0) {
        tau = 0.0;
        return;
    }
    double xnorm = dznrm2(n - 1, x, incx);
    double alphr = alpha.real(), alphi = alpha.imag();
    if (xnorm == 0.0 && alphi == 0.0) {
        tau = 0.0;
        return;
    }
    double beta = -std::copysign(dlapy3(alphr, alphi, xnorm), alphr);
    const double safmin = kSafmin / la::kEps, rsafmn = 1.0 / safmin;
    int knt = 0;
    if (std::fabs(beta) < safmin) {
        do {
            ++knt;
            for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= rsafmn;
            beta *= rsafmn;
            alphi *= rsafmn;
            alphr *= rsafmn;
        } while (std::fabs(beta) < safmin && knt < 20);
        xnorm = dznrm2(n - 1, x, incx);
        alpha = cd(alphr, alphi);
        beta = -std::copysign(dlapy3(alphr, alphi, xnorm), alphr);
    }
    tau = cd((beta - alphr) / beta, -alphi / beta);
    alpha = cdiv(cd(1.0), alpha - beta);
    for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= alpha;
    for (int j = 0; j < knt; ++j) beta *= safmin;
    alpha = beta;
}

void larf(char side, int m, int n, const cd* v, cd tau, cd* c, int ldc, cd* work) {
    if (tau == cd(0.0)) return;
    if (side == 'L') {  // w = C^H v ; C -= tau v w^H
        for (int j = 0; j < n; ++j) {
            cd s = 0.0;
            for (int i = 0; i < m; ++i) s += std::conj(c[i + (size_t)j * ldc]) * v[i];
            work[j] = s;
        }
        for (int j = 0; j < n; ++j) {
            const cd t = -tau * std::conj(work[j]);
            for (int i = 0; i < m; ++i) c[i + (size_t)j * ldc] += v[i] * t;
        }
    } else {  // w = C v ; C -= tau w v^H
        for (int i = 0; i < m; ++i) work[i] = 0.0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i) work[i] += c[i + (size_t)j * ldc] * v[j];
        for (int j = 0; j < n; ++j) {
            const cd t = -tau * std::conj(v[j]);
            for (int i = 0; i < m; ++i) c[i + (size_t)j * ldc] += work[i] * t;
        }
    }
}

void geqr2(int m, int n, cd* a, int lda, cd* tau, cd* work) {
    const int k = std::min(m, n);
    for (int i = 0; i < k; ++i) {
        cd* aii = a + i + (size_t)i * lda;
        larfg(m - i, *aii, a + std::min(i + 1, m - 1) + (size_t)i * lda, 1, tau[i]);
        if (i < n - 1) {
            const cd keep = *aii;
            *aii = 1.0;
            larf('L', m - i, n - i - 1, aii, std::conj(tau[i]), a + i + (size_t)(i + 1) * lda, lda, work);
            *aii = keep;
        }
    }
}

void unm2r_rn(int m, int n, int k, cd* a, int lda, const cd* tau, cd* c, int ldc, cd* work) {
    for (int i = 0; i < k; ++i) {  // C := C * H_i, i = 1..k, on columns i..n
        cd* aii = a + i + (size_t)i * lda;
        const cd keep = *aii;
        *aii = 1.0;
        larf('R', m, n - i, aii, tau[i], c + (size_t)i * ldc, ldc, work);
        *aii = keep;
    }
}

void unm2r_ln(int m, int n, int k, cd* a, int lda, const cd* tau, cd* c, int ldc, cd* work) {
    for (int i = k - 1; i >= 0; --i) {  // C := H_i * C, i = k..1, on rows i..m
        cd* aii = a + i + (size_t)i * lda;
        const cd keep = *aii;
        *aii = 1.0;
        larf('L', m - i, n, aii, tau[i], c + i, ldc, work);
        *aii = keep;
    }
}

int lahqr(bool wantt, bool wantz, int n, int ilo, int ihi, cd* h, int ldh, cd* w, int iloz,
          int ihiz, cd* z, int ldz) {
#define H(i, j) h[((i)-1) + (size_t)((j)-1) * ldh]
#define Z(i, j) z[((i)-1) + (size_t)((j)-1) * ldz]
    const double dat1 = 3.0 / 4.0;
    const int kexsh = 10;
    if (n == 0) return 0;
    if (ilo == ihi) {
        w[ilo - 1] = H(ilo, ilo);
        return 0;
    }
    for (int j = ilo; j <= ihi - 3; ++j) {
        H(j + 2, j) = 0.0;
        H(j + 3, j) = 0.0;
    }
    if (ilo <= ihi - 2) H(ihi, ihi - 2) = 0.0;
    const int jlo = wantt ? 1 : ilo, jhi = wantt ? n : ihi;
    for (int i = ilo + 1; i <= ihi; ++i) {  // make the subdiagonal real
        if (H(i, i - 1).imag() != 0.0) {
            cd sc = H(i, i - 1) / cabs1(H(i, i - 1));
            sc = std::conj(sc) / std::abs(sc);
            H(i, i - 1) = std::abs(H(i, i - 1));
            for (int j = i; j <= jhi; ++j) H(i, j) *= sc;
            for (int j = jlo; j <= std::min(jhi, i + 1); ++j) H(j, i) *= std::conj(sc);
            if (wantz)
                for (int j = iloz; j <= ihiz; ++j) Z(j, i) *= std::conj(sc);
        }
    }
    const int nh = ihi - ilo + 1, nz = ihiz - iloz + 1;
    const double safmin = kSafmin, ulp = kUlp;
    const double smlnum = safmin * ((double)nh / ulp);
    int i1 = 1, i2 = n;
    const int itmax = 30 * std::max(10, nh);
    int kdefl = 0;
    int i = ihi;
    cd v[2];
    for (;;) {
        if (i < ilo) return 0;
        int l = ilo;
        bool conv = false;
        for (int its = 0; its <= itmax; ++its) {
            int k;
            for (k = i; k >= l + 1; --k) {
                if (cabs1(H(k, k - 1)) <= smlnum) break;
                double tst = cabs1(H(k - 1, k - 1)) + cabs1(H(k, k));
                if (tst == 0.0) {
                    if (k - 2 >= ilo) tst += std::fabs(H(k - 1, k - 2).real());
                    if (k + 1 <= ihi) tst += std::fabs(H(k + 1, k).real());
                }
                if (std::fabs(H(k, k - 1).real()) <= ulp * tst) {
                    const double ab = std::max(cabs1(H(k, k - 1)), cabs1(H(k - 1, k)));
                    const double ba = std::min(cabs1(H(k, k - 1)), cabs1(H(k - 1, k)));
                    const double aa = std::max(cabs1(H(k, k)), cabs1(H(k - 1, k - 1) - H(k, k)));
                    const double bb = std::min(cabs1(H(k, k)), cabs1(H(k - 1, k - 1) - H(k, k)));
                    const double s = aa + ab;
                    if (ba * (ab / s) <= std::max(smlnum, ulp * (bb * (aa / s)))) break;
                }
            }
            l = k;
            if (l > ilo) H(l, l - 1) = 0.0;
            if (l >= i) {
                conv = true;
                break;
            }
            ++kdefl;
            if (!wantt) {
                i1 = l;
                i2 = i;
            }
            cd t;
            if (kdefl % (2 * kexsh) == 0) {
                const double s = dat1 * std::fabs(H(i, i - 1).real());
                t = s + H(i, i);
            } else if (kdefl % kexsh == 0) {
                const double s = dat1 * std::fabs(H(l + 1, l).real());
                t = s + H(l, l);
            } else {  // Wilkinson's shift
                t = H(i, i);
                const cd u = std::sqrt(H(i - 1, i)) * std::sqrt(H(i, i - 1));
                double s = cabs1(u);
                if (s != 0.0) {
                    const cd x = 0.5 * (H(i - 1, i - 1) - t);
                    const double sx = cabs1(x);
                    s = std::max(s, cabs1(x));
                    const cd xs = x / s, us = u / s;
                    cd y = s * std::sqrt(xs * xs + us * us);
                    if (sx > 0.0) {
                        const cd xsx = x / sx;
                        if (xsx.real() * y.real() + xsx.imag() * y.imag() < 0.0) y = -y;
                    }
                    t = t - u * cdiv(u, x + y);
                }
            }
            int m;
            cd h11, h22, h11s;
            double h21;
            for (m = i - 1; m >= l + 1; --m) {
                h11 = H(m, m);
                h22 = H(m + 1, m + 1);
                h11s = h11 - t;
                h21 = H(m + 1, m).real();
                const double s = cabs1(h11s) + std::fabs(h21);
                h11s /= s;
                h21 /= s;
                v[0] = h11s;
                v[1] = h21;
                const double h10 = H(m, m - 1).real();
                if (std::fabs(h10) * std::fabs(h21) <= ulp * (cabs1(h11s) * (cabs1(h11) + cabs1(h22)))) break;
            }
            if (m == l) {
                h11 = H(l, l);
                h22 = H(l + 1, l + 1);
                h11s = h11 - t;
                h21 = H(l + 1, l).real();
                const double s = cabs1(h11s) + std::fabs(h21);
                h11s /= s;
                h21 /= s;
                v[0] = h11s;
                v[1] = h21;
            }
            for (int kk = m; kk <= i - 1; ++kk) {
                if (kk > m) {
                    v[0] = H(kk, kk - 1);
                    v[1] = H(kk + 1, kk - 1);
                }
                cd t1;
                larfg(2, v[0], v + 1, 1, t1);
                if (kk > m) {
                    H(kk, kk - 1) = v[0];
                    H(kk + 1, kk - 1) = 0.0;
                }
                const cd v2 = v[1];
                const double t2 = (t1 * v2).real();
                for (int j = kk; j <= i2; ++j) {
                    const cd sum = std::conj(t1) * H(kk, j) + t2 * H(kk + 1, j);
                    H(kk, j) -= sum;
                    H(kk + 1, j) -= sum * v2;
                }
                for (int j = i1; j <= std::min(kk + 2, i); ++j) {
                    const cd sum = t1 * H(j, kk) + t2 * H(j, kk + 1);
                    H(j, kk) -= sum;
                    H(j, kk + 1) -= sum * std::conj(v2);
                }
                if (wantz) {
                    for (int j = iloz; j <= ihiz; ++j) {
                        const cd sum = t1 * Z(j, kk) + t2 * Z(j, kk + 1);
                        Z(j, kk) -= sum;
                        Z(j, kk + 1) -= sum * std::conj(v2);
                    }
                }
                if (kk == m && m > l) {
                    cd temp = 1.0 - t1;
                    temp /= std::abs(temp);
                    H(m + 1, m) *= std::conj(temp);
                    if (m + 2 <= i) H(m + 2, m + 1) *= temp;
                    for (int j = m; j <= i; ++j) {
                        if (j != m + 1) {
                            if (i2 > j)
                                for (int c = j + 1; c <= i2; ++c) H(j, c) *= temp;
                            for (int r = i1; r <= j - 1; ++r) H(r, j) *= std::conj(temp);
                            if (wantz)
                                for (int r = iloz; r < iloz + nz; ++r) Z(r, j) *= std::conj(temp);
                        }
                    }
                }
            }
            cd temp = H(i, i - 1);
            if (temp.imag() != 0.0) {
                const double rtemp = std::abs(temp);
                H(i, i - 1) = rtemp;
                temp /= rtemp;
                if (i2 > i)
                    for (int c = i + 1; c <= i2; ++c) H(i, c) *= std::conj(temp);
                for (int r = i1; r <= i - 1; ++r) H(r, i) *= temp;
                if (wantz)
                    for (int r = iloz; r < iloz + nz; ++r) Z(r, i) *= temp;
            }
        }
        if (!conv) return i;
        w[i - 1] = H(i, i);
        kdefl = 0;
        i = l - 1;
    }
#undef H
#undef Z
}

int trevc_right(char howmny, int* select, int n, cd* t, int ldt, cd* vr, int ldvr, cd* work) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
#define VR(i, j) vr[((i)-1) + (size_t)((j)-1) * ldvr]
    const bool over = howmny == 'B', somev = howmny == 'S';
    int m = n;
    if (somev) {
        m = 0;
        for (int j = 0; j < n; ++j)
            if (select[j]) ++m;
    }
    if (n == 0) return m;
    const double unfl = kSafmin, ulp = kUlp;
    const double smlnum = unfl * (n / ulp);
    std::vector<cd> diag(n);
    for (int i = 1; i <= n; ++i) diag[i - 1] = T(i, i);
    int is = m;
    for (int ki = n; ki >= 1; --ki) {
        if (somev && !select[ki - 1]) continue;
        const double smin = std::max(ulp * cabs1(T(ki, ki)), smlnum);
        work[0] = 1.0;
        for (int k = 1; k <= ki - 1; ++k) work[k - 1] = -T(k, ki);
        for (int k = 1; k <= ki - 1; ++k) {
            T(k, k) = T(k, k) - T(ki, ki);
            if (cabs1(T(k, k)) < smin) T(k, k) = smin;
        }
        double scale = 1.0;
        if (ki > 1) {  // zlatrs('U','N','N','Y') in its unscaled (ztrsv) regime
            for (int j = ki - 1; j >= 1; --j) {
                if (work[j - 1] != cd(0.0)) {
                    work[j - 1] = cdiv(work[j - 1], T(j, j));
                    const cd tmp = work[j - 1];
                    for (int r = j - 1; r >= 1; --r) work[r - 1] -= tmp * T(r, j);
                }
            }
            work[ki - 1] = scale;
        }
        if (!over) {
            for (int k = 1; k <= ki; ++k) VR(k, is) = work[k - 1];
            int ii = 1;
            double best = cabs1(VR(1, is));
            for (int k = 2; k <= ki; ++k)
                if (cabs1(VR(k, is)) > best) {
                    best = cabs1(VR(k, is));
                    ii = k;
                }
            const double remax = 1.0 / cabs1(VR(ii, is));
            for (int k = 1; k <= ki; ++k) VR(k, is) *= remax;
            for (int k = ki + 1; k <= n; ++k) VR(k, is) = 0.0;
        } else {
            if (ki > 1) {  // zgemv('N', n, ki-1, 1, VR, work, scale, VR(:,ki))
                for (int r = 1; r <= n; ++r) VR(r, ki) *= scale;
                for (int c = 1; c <= ki - 1; ++c) {
                    const cd tmp = work[c - 1];
                    for (int r = 1; r <= n; ++r) VR(r, ki) += tmp * VR(r, c);
                }
            }
            int ii = 1;
            double best = cabs1(VR(1, ki));
            for (int k = 2; k <= n; ++k)
                if (cabs1(VR(k, ki)) > best) {
                    best = cabs1(VR(k, ki));
                    ii = k;
                }
            const double remax = 1.0 / cabs1(VR(ii, ki));
            for (int k = 1; k <= n; ++k) VR(k, ki) *= remax;
        }
        for (int k = 1; k <= ki - 1; ++k) T(k, k) = diag[k - 1];
        --is;
    }
    return m;
#undef T
#undef VR
}

int trsen(const int* select, int n, cd* t, int ldt, cd* q, int ldq, cd* w, int& m) {
#define T(i, j) t[((i)-1) + (size_t)((j)-1) * ldt]
#define Q(i, j) q[((i)-1) + (size_t)((j)-1) * ldq]
    m = 0;
    for (int k = 0; k < n; ++k)
        if (select[k]) ++m;
    if (!(m == n || m == 0)) {
        int ks = 0;
        for (int k = 1; k <= n; ++k) {
            if (!select[k - 1]) continue;
            ++ks;
            if (k != ks) {  // ztrexc(compq='V', ifst=k, ilst=ks): adjacent swaps upwards
                for (int kk = k - 1; kk >= ks; --kk) {
                    const cd t11 = T(kk, kk), t22 = T(kk + 1, kk + 1);
                    double cs;
                    cd sn, temp;
                    lartg(T(kk, kk + 1), t22 - t11, cs, sn, temp);
                    if (kk + 2 <= n) zrot(n - kk - 1, &T(kk, kk + 2), ldt, &T(kk + 1, kk + 2), ldt, cs, sn);
                    zrot(kk - 1, &T(1, kk), 1, &T(1, kk + 1), 1, cs, std::conj(sn));
                    T(kk, kk) = t22;
                    T(kk + 1, kk + 1) = t11;
                    zrot(n, &Q(1, kk), 1, &Q(1, kk + 1), 1, cs, std::conj(sn));
                }
            }
        }
    }
    for (int k = 1; k <= n; ++k) w[k - 1] = T(k, k);
    return 0;
#undef T
#undef Q
}

// ---------------------------------------------------------------- ARPACK ----
void zsortc(Which which, bool apply, int n, cd* x, cd* y) {
    auto ooo = [&](int a, int b) -> bool {
        switch (which) {
            case Which::LM: return la::lapy2(x[a].real(), x[a].imag()) > la::lapy2(x[b].real(), x[b].imag());
            case Which::SM: return la::lapy2(x[a].real(), x[a].imag()) < la::lapy2(x[b].real(), x[b].imag());
            case Which::LR: return x[a].real() > x[b].real();
            case Which::SR: return x[a].real() < x[b].real();
            case Which::LI: return x[a].imag() > x[b].imag();
            case Which::SI: return x[a].imag() < x[b].imag();
            default: return false;
        }
    };
    for (int igap = n / 2; igap != 0; igap /= 2)
        for (int i = igap; i <= n - 1; ++i)
            for (int j = i - igap; j >= 0; j -= igap) {
                if (!ooo(j, j + igap)) break;
                std::swap(x[j], x[j + igap]);
                if (apply) std::swap(y[j], y[j + igap]);
            }
}

void zngets(int ishift, Which which, int kev, int np, cd* ritz, cd* bounds) {
    zsortc(which, true, kev + np, ritz, bounds);
    if (ishift == 1) zsortc(Which::SM, true, np, bounds, ritz);
}

int zneigh(double rnorm, int n, const cd* h, int ldh, cd* ritz, cd* bounds, cd* q, int ldq,
           cd* workl) {
    for (int j = 0; j < n; ++j) std::memcpy(workl + (size_t)j * n, h + (size_t)j * ldh, sizeof(cd) * n);
    for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) q[i + (size_t)j * ldq] = (i == j) ? 1.0 : 0.0;
    // the reference passes ldh as the leading dimension of its n x n copy (zneigh.f:176)
    int ierr = lahqr(true, true, n, 1, n, workl, ldh, ritz, 1, n, q, ldq);
    if (ierr != 0) return ierr;
    std::vector<int> sel(n, 0);
    trevc_right('B', sel.data(), n, workl, n, q, ldq, workl + (size_t)n * n);
    for (int j = 0; j < n; ++j) {
        const double s = 1.0 / dznrm2(n, q + (size_t)j * ldq, 1);
        for (int r = 0; r < n; ++r) q[r + (size_t)j * ldq] *= s;
    }
    for (int j = 0; j < n; ++j) bounds[j] = q[(n - 1) + (size_t)j * n] * rnorm;
    return 0;
}

void znapps_host(int kev, int np, const cd* shift, cd* h, int ldh, cd* q, int ldq, cd* workl,
                 int64_t nglob) {
#define H(i, j) h[((i)-1) + (size_t)((j)-1) * ldh]
#define Q(i, j) q[((i)-1) + (size_t)((j)-1) * ldq]
    const double ulp = kUlp, smlnum = kSafmin * ((double)nglob / ulp);
    const int kplusp = kev + np;
    for (int j = 1; j <= kplusp; ++j)
        for (int i = 1; i <= kplusp; ++i) Q(i, j) = (i == j) ? 1.0 : 0.0;
    (void)workl;
    if (np == 0) return;
    for (int jj = 1; jj <= np; ++jj) {
        const cd sigma = shift[jj - 1];
        int istart = 1;
        for (;;) {
            int iend = kplusp;
            for (int i = istart; i <= kplusp - 1; ++i) {
                double tst1 = cabs1(H(i, i)) + cabs1(H(i + 1, i + 1));
                if (tst1 == 0.0) tst1 = lanhs1(kplusp - jj + 1, h, ldh);
                if (std::fabs(H(i + 1, i).real()) <= std::max(ulp * tst1, smlnum)) {
                    iend = i;
                    H(i + 1, i) = 0.0;
                    break;
                }
            }
            if (!(istart == iend || istart > kev)) {
                cd f = H(istart, istart) - sigma, g = H(istart + 1, istart);
                for (int i = istart; i <= iend - 1; ++i) {
                    double c;
                    cd s, r;
                    lartg(f, g, c, s, r);
                    if (i > istart) {
                        H(i, i - 1) = r;
                        H(i + 1, i - 1) = 0.0;
                    }
                    for (int j = i; j <= kplusp; ++j) {
                        const cd t = c * H(i, j) + s * H(i + 1, j);
                        H(i + 1, j) = -std::conj(s) * H(i, j) + c * H(i + 1, j);
                        H(i, j) = t;
                    }
                    for (int j = 1; j <= std::min(i + 2, iend); ++j) {
                        const cd t = c * H(j, i) + std::conj(s) * H(j, i + 1);
                        H(j, i + 1) = -s * H(j, i) + c * H(j, i + 1);
                        H(j, i) = t;
                    }
                    for (int j = 1; j <= std::min(i + jj, kplusp); ++j) {
                        const cd t = c * Q(j, i) + std::conj(s) * Q(j, i + 1);
                        Q(j, i + 1) = -s * Q(j, i) + c * Q(j, i + 1);
                        Q(j, i) = t;
                    }
                    if (i < iend - 1) {
                        f = H(i + 1, i);
                        g = H(i + 2, i);
                    }
                }
            }
            istart = iend + 1;
            if (iend >= kplusp) break;
        }
    }
    for (int j = 1; j <= kev; ++j) {  // real non-negative subdiagonal (SRC/znapps.f:453-462)
        if (H(j + 1, j).real() < 0.0 || H(j + 1, j).imag() != 0.0) {
            const cd t = H(j + 1, j) / la::lapy2(H(j + 1, j).real(), H(j + 1, j).imag());
            for (int c = j; c <= kplusp; ++c) H(j + 1, c) *= std::conj(t);
            for (int r = 1; r <= std::min(j + 2, kplusp); ++r) H(r, j + 1) *= t;
            for (int r = 1; r <= std::min(j + np + 1, kplusp); ++r) Q(r, j + 1) *= t;
            H(j + 1, j) = cd(H(j + 1, j).real(), 0.0);
        }
    }
    for (int i = 1; i <= kev; ++i) {
        double tst1 = cabs1(H(i, i)) + cabs1(H(i + 1, i + 1));
        if (tst1 == 0.0) tst1 = lanhs1(kev, h, ldh);
        if (H(i + 1, i).real() <= std::max(ulp * tst1, smlnum)) H(i + 1, i) = 0.0;
    }
#undef H
#undef Q
}

}  // namespace ahip::zla
