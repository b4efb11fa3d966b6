// Host small-dense kit — see dense.hpp.  Indices inside the LAPACK-derived
// routines are kept 1-based through small accessor lambdas so the published
// algorithms can be checked line by line against their descriptions.
#include "dense.hpp"

#include <algorithm>
#include <cstring>

namespace ahip::la {

namespace {
inline double sign(double a, double b) { return std::signbit(b) ? -std::fabs(a) : std::fabs(a); }
}  // namespace

double lapy2(double x, double y) {
    if (std::isnan(x)) return x;
    if (std::isnan(y)) return y;
    const double xa = std::fabs(x), ya = std::fabs(y);
    const double w = std::max(xa, ya), z = std::min(xa, ya);
    if (z == 0.0 || w > DBL_MAX) return w;
    const double q = z / w;
    return w * std::sqrt(1.0 + q * q);
}

void lartg(double f, double g, double& c, double& s, double& r) {
    const double safmin = kSafmin, safmax = 1.0 / kSafmin;
    const double rtmin = std::sqrt(safmin), rtmax = std::sqrt(safmax / 2);
    const double f1 = std::fabs(f), g1 = std::fabs(g);
    if (g == 0.0) {
        c = 1.0; s = 0.0; r = f;
    } else if (f == 0.0) {
        c = 0.0; s = sign(1.0, g); r = g1;
    } else if (f1 > rtmin && f1 < rtmax && g1 > rtmin && g1 < rtmax) {
        const double d = std::sqrt(f * f + g * g);
        c = f1 / d;
        r = sign(d, f);
        s = g / r;
    } else {
        const double u = std::min(safmax, std::max(safmin, std::max(f1, g1)));
        const double fs = f / u, gs = g / u;
        const double d = std::sqrt(fs * fs + gs * gs);
        c = std::fabs(fs) / d;
        r = sign(d, f);
        s = gs / r;
        r *= u;
    }
}

// Eigen-decomposition of the 2x2 symmetric [[a,b],[b,c]] (dlae2 / dlaev2).
static void two_by_two(double a, double b, double c, double& rt1, double& rt2,
                       double* cs1, double* sn1) {
    const double sm = a + c, df = a - c, adf = std::fabs(df), tb = b + b, ab = std::fabs(tb);
    double acmx, acmn;
    if (std::fabs(a) > std::fabs(c)) { acmx = a; acmn = c; } else { acmx = c; acmn = a; }
    double rt;
    if (adf > ab) { const double q = ab / adf; rt = adf * std::sqrt(1.0 + q * q); }
    else if (adf < ab) { const double q = adf / ab; rt = ab * std::sqrt(1.0 + q * q); }
    else rt = ab * std::sqrt(2.0);
    int sgn1;
    if (sm < 0.0) {
        rt1 = 0.5 * (sm - rt); sgn1 = -1;
        rt2 = (acmx / rt1) * acmn - (b / rt1) * b;
    } else if (sm > 0.0) {
        rt1 = 0.5 * (sm + rt); sgn1 = 1;
        rt2 = (acmx / rt1) * acmn - (b / rt1) * b;
    } else {
        rt1 = 0.5 * rt; rt2 = -0.5 * rt; sgn1 = 1;
    }
    if (!cs1) return;
    int sgn2;
    double cs;
    if (df >= 0.0) { cs = df + rt; sgn2 = 1; } else { cs = df - rt; sgn2 = -1; }
    const double acs = std::fabs(cs);
    if (acs > ab) {
        const double ct = -tb / cs;
        *sn1 = 1.0 / std::sqrt(1.0 + ct * ct);
        *cs1 = ct * *sn1;
    } else if (ab == 0.0) {
        *cs1 = 1.0; *sn1 = 0.0;
    } else {
        const double tn = -cs / tb;
        *cs1 = 1.0 / std::sqrt(1.0 + tn * tn);
        *sn1 = tn * *cs1;
    }
    if (sgn1 == sgn2) { const double tn = *cs1; *cs1 = -*sn1; *sn1 = tn; }
}

void lae2(double a, double b, double c, double& rt1, double& rt2) {
    two_by_two(a, b, c, rt1, rt2, nullptr, nullptr);
}
void laev2(double a, double b, double c, double& rt1, double& rt2, double& cs1, double& sn1) {
    two_by_two(a, b, c, rt1, rt2, &cs1, &sn1);
}

int lascl_factors(double cfrom, double cto, double mul[4]) {
    const double smlnum = kSafmin, bignum = 1.0 / smlnum;
    double cfromc = cfrom, ctoc = cto;
    int k = 0;
    for (;;) {
        const double cfrom1 = cfromc * smlnum;
        double m;
        bool done;
        if (cfrom1 == cfromc) {  // cfromc is inf: result is a NaN/0 pattern, as LAPACK
            m = ctoc / cfromc; done = true;
        } else {
            const double cto1 = ctoc / bignum;
            if (cto1 == ctoc) { m = ctoc; done = true; cfromc = 1.0; }
            else if (std::fabs(cfrom1) > std::fabs(ctoc) && ctoc != 0.0) {
                m = smlnum; done = false; cfromc = cfrom1;
            } else if (std::fabs(cto1) > std::fabs(cfromc)) {
                m = bignum; done = false; ctoc = cto1;
            } else { m = ctoc / cfromc; done = true; }
        }
        mul[k++] = m;
        if (done || k == 4) return k;
    }
}

void lascl(double cfrom, double cto, int n, double* x) {
    double mul[4];
    const int k = lascl_factors(cfrom, cto, mul);
    for (int t = 0; t < k; ++t)
        for (int i = 0; i < n; ++i) x[i] *= mul[t];
}

// Apply the plane rotations (c_j, s_j), j = 1..nn-1, from the right to the
// `rows` x nn block Z (dlasr side='R', pivot='V').  backward: j = nn-1 .. 1.
static void rot_right(int rows, int nn, const double* c, const double* s, double* z,
                      int ldz, bool backward) {
    auto body = [&](int j) {  // 1-based j
        const double ct = c[j - 1], st = s[j - 1];
        if (ct == 1.0 && st == 0.0) return;
        double* zj = z + (size_t)(j - 1) * ldz;
        double* zj1 = z + (size_t)j * ldz;
        for (int i = 0; i < rows; ++i) {
            const double t = zj1[i];
            zj1[i] = ct * t - st * zj[i];
            zj[i] = st * t + ct * zj[i];
        }
    };
    if (backward) for (int j = nn - 1; j >= 1; --j) body(j);
    else for (int j = 1; j <= nn - 1; ++j) body(j);
}

int steqr(int n, double* dd, double* ee, double* zz, int zrows, int ldz, double* work,
          bool one_norm_inf) {
    // 1-based views
    auto D = [&](int i) -> double& { return dd[i - 1]; };
    auto E = [&](int i) -> double& { return ee[i - 1]; };
    auto Zc = [&](int j) -> double* { return zz + (size_t)(j - 1) * ldz; };  // column j
    auto W = [&](int i) -> double& { return work[i - 1]; };
    int info = 0;
    if (n == 0) return 0;
    // Z := identity rows (all of I for dsteqr, its last row for dstqrb)
    for (int j = 1; j <= n; ++j)
        for (int i = 0; i < zrows; ++i)
            Zc(j)[i] = (zrows == 1) ? (j == n ? 1.0 : 0.0) : (i == j - 1 ? 1.0 : 0.0);
    if (n == 1) return 0;

    const double eps = kEps, eps2 = eps * eps, safmin = kSafmin, safmax = 1.0 / safmin;
    const double ssfmax = std::sqrt(safmax) / 3.0, ssfmin = std::sqrt(safmin) / eps2;
    const int maxit = 30, nmaxit = n * maxit;
    int jtot = 0, l1 = 1;
    const int nm1 = n - 1;

    auto tri_norm = [&](int l, int lend) {
        const int m = lend - l + 1;
        double a = 0.0;
        if (!one_norm_inf) {  // 'M': max abs
            for (int i = 0; i < m; ++i) a = std::max(a, std::fabs(D(l + i)));
            for (int i = 0; i < m - 1; ++i) a = std::max(a, std::fabs(E(l + i)));
        } else if (m == 1) {
            a = std::fabs(D(l));
        } else {  // 'I' (== '1' for symmetric): max row sum
            a = std::max(std::fabs(D(l)) + std::fabs(E(l)),
                         std::fabs(E(l + m - 2)) + std::fabs(D(l + m - 1)));
            for (int i = 1; i < m - 1; ++i)
                a = std::max(a, std::fabs(D(l + i)) + std::fabs(E(l + i)) +
                                    std::fabs(E(l + i - 1)));
        }
        return a;
    };

    for (;;) {  // label 10
        if (l1 > n) break;  // -> 160 (sort)
        if (l1 > 1) E(l1 - 1) = 0.0;
        int m = n;
        if (l1 <= nm1) {
            for (int mm = l1; mm <= nm1; ++mm) {
                const double tst = std::fabs(E(mm));
                if (tst == 0.0) { m = mm; break; }
                if (tst <= (std::sqrt(std::fabs(D(mm))) * std::sqrt(std::fabs(D(mm + 1)))) * eps) {
                    E(mm) = 0.0; m = mm; break;
                }
            }
        }
        int l = l1;
        const int lsv = l;
        int lend = m;
        const int lendsv = lend;
        l1 = m + 1;
        if (lend == l) continue;
        const double anorm = tri_norm(l, lend);
        int iscale = 0;
        if (anorm == 0.0) continue;
        if (anorm > ssfmax) {
            iscale = 1;
            lascl(anorm, ssfmax, lend - l + 1, &D(l));
            lascl(anorm, ssfmax, lend - l, &E(l));
        } else if (anorm < ssfmin) {
            iscale = 2;
            lascl(anorm, ssfmin, lend - l + 1, &D(l));
            lascl(anorm, ssfmin, lend - l, &E(l));
        }
        if (std::fabs(D(lend)) < std::fabs(D(l))) { lend = lsv; l = lendsv; }

        if (lend > l) {
            // QL iteration: look for a small subdiagonal element (label 40)
            for (;;) {
                int mq = lend;
                if (l != lend) {
                    for (int k = l; k <= lend - 1; ++k) {
                        const double tst = std::fabs(E(k)) * std::fabs(E(k));
                        if (tst <= (eps2 * std::fabs(D(k))) * std::fabs(D(k + 1)) + safmin) {
                            mq = k; break;
                        }
                    }
                }
                if (mq < lend) E(mq) = 0.0;
                double p = D(l);
                if (mq == l) {  // label 80: eigenvalue found
                    D(l) = p;
                    ++l;
                    if (l <= lend) continue;
                    break;
                }
                if (mq == l + 1) {  // 2x2 block
                    double rt1, rt2, c, s;
                    laev2(D(l), E(l), D(l + 1), rt1, rt2, c, s);
                    W(l) = c; W(n - 1 + l) = s;
                    rot_right(zrows, 2, &W(l), &W(n - 1 + l), Zc(l), ldz, true);
                    D(l) = rt1; D(l + 1) = rt2; E(l) = 0.0;
                    l += 2;
                    if (l <= lend) continue;
                    break;
                }
                if (jtot == nmaxit) break;
                ++jtot;
                double g = (D(l + 1) - p) / (2.0 * E(l));
                double r = lapy2(g, 1.0);
                g = D(mq) - p + (E(l) / (g + sign(r, g)));
                double s = 1.0, c = 1.0;
                p = 0.0;
                for (int i = mq - 1; i >= l; --i) {
                    const double f = s * E(i), b = c * E(i);
                    lartg(g, f, c, s, r);
                    if (i != mq - 1) E(i + 1) = r;
                    g = D(i + 1) - p;
                    r = (D(i) - g) * s + 2.0 * c * b;
                    p = s * r;
                    D(i + 1) = g + p;
                    g = c * r - b;
                    W(i) = c; W(n - 1 + i) = -s;
                }
                rot_right(zrows, mq - l + 1, &W(l), &W(n - 1 + l), Zc(l), ldz, true);
                D(l) = D(l) - p;
                E(l) = g;
            }
        } else {
            // QR iteration (label 90)
            for (;;) {
                int mq = lend;
                if (l != lend) {
                    for (int k = l; k >= lend + 1; --k) {
                        const double tst = std::fabs(E(k - 1)) * std::fabs(E(k - 1));
                        if (tst <= (eps2 * std::fabs(D(k))) * std::fabs(D(k - 1)) + safmin) {
                            mq = k; break;
                        }
                    }
                }
                if (mq > lend) E(mq - 1) = 0.0;
                double p = D(l);
                if (mq == l) {  // label 130
                    D(l) = p;
                    --l;
                    if (l >= lend) continue;
                    break;
                }
                if (mq == l - 1) {
                    double rt1, rt2, c, s;
                    laev2(D(l - 1), E(l - 1), D(l), rt1, rt2, c, s);
                    W(mq) = c; W(n - 1 + mq) = s;
                    rot_right(zrows, 2, &W(mq), &W(n - 1 + mq), Zc(l - 1), ldz, false);
                    D(l - 1) = rt1; D(l) = rt2; E(l - 1) = 0.0;
                    l -= 2;
                    if (l >= lend) continue;
                    break;
                }
                if (jtot == nmaxit) break;
                ++jtot;
                double g = (D(l - 1) - p) / (2.0 * E(l - 1));
                double r = lapy2(g, 1.0);
                g = D(mq) - p + (E(l - 1) / (g + sign(r, g)));
                double s = 1.0, c = 1.0;
                p = 0.0;
                for (int i = mq; i <= l - 1; ++i) {
                    const double f = s * E(i), b = c * E(i);
                    lartg(g, f, c, s, r);
                    if (i != mq) E(i - 1) = r;
                    g = D(i) - p;
                    r = (D(i + 1) - g) * s + 2.0 * c * b;
                    p = s * r;
                    D(i) = g + p;
                    g = c * r - b;
                    W(i) = c; W(n - 1 + i) = s;
                }
                rot_right(zrows, l - mq + 1, &W(mq), &W(n - 1 + mq), Zc(mq), ldz, false);
                D(l) = D(l) - p;
                E(l - 1) = g;
            }
        }
        // label 140: undo scaling
        if (iscale == 1) {
            lascl(ssfmax, anorm, lendsv - lsv + 1, &D(lsv));
            lascl(ssfmax, anorm, lendsv - lsv, &E(lsv));
        } else if (iscale == 2) {
            lascl(ssfmin, anorm, lendsv - lsv + 1, &D(lsv));
            lascl(ssfmin, anorm, lendsv - lsv, &E(lsv));
        }
        if (jtot >= nmaxit) {
            for (int i = 1; i <= n - 1; ++i)
                if (E(i) != 0.0) ++info;
            return info;
        }
    }
    // label 160: selection sort into increasing order, permuting Z columns
    for (int ii = 2; ii <= n; ++ii) {
        const int i = ii - 1;
        int k = i;
        double p = D(i);
        for (int j = ii; j <= n; ++j)
            if (D(j) < p) { k = j; p = D(j); }
        if (k != i) {
            D(k) = D(i);
            D(i) = p;
            for (int r = 0; r < zrows; ++r) std::swap(Zc(i)[r], Zc(k)[r]);
        }
    }
    return info;
}

// dnrm2 as the image's OpenBLAS computes it (x86-64 kernel: sum of squares in
// x87 extended precision, one rounding at the end) -- bit-identical on 2,700
// random vectors (tests/test_kit_ns.py), which the scaled LAPACK reference
// algorithm is not.
double nrm2(int n, const double* x, int incx) {
    if (n < 1) return 0.0;
    long double s = 0.0L;
    for (int i = 0; i < n; ++i) {
        const long double v = x[(size_t)i * incx];
        s += v * v;
    }
    return (double)std::sqrt(s);
}

void larfg(int n, double& alpha, double* x, int incx, double& tau) {
    if (n <= 1) { tau = 0.0; return; }
    double xnorm = nrm2(n - 1, x, incx);
    if (xnorm == 0.0) { tau = 0.0; return; }
    double beta = -sign(lapy2(alpha, xnorm), alpha);
    const double safmin = kSafmin / kEps;
    int knt = 0;
    if (std::fabs(beta) < safmin) {
        const double rsafmn = 1.0 / safmin;
        do {
            ++knt;
            for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= rsafmn;
            beta *= rsafmn;
            alpha *= rsafmn;
        } while (std::fabs(beta) < safmin && knt < 20);
        xnorm = nrm2(n - 1, x, incx);
        beta = -sign(lapy2(alpha, xnorm), alpha);
    }
    tau = (beta - alpha) / beta;
    const double sc = 1.0 / (alpha - beta);
    for (int i = 0; i < n - 1; ++i) x[(size_t)i * incx] *= sc;
    for (int j = 0; j < knt; ++j) beta *= safmin;
    alpha = beta;
}

void larf(char side, int m, int n, const double* v, int incv, double tau, double* c, int ldc,
          double* work) {
    if (tau == 0.0) return;
    if (side == 'L') {  // C := (I - tau v v^T) C ; w = C^T v
        for (int j = 0; j < n; ++j) {
            double s = 0.0;
            for (int i = 0; i < m; ++i) s += c[i + (size_t)j * ldc] * v[(size_t)i * incv];
            work[j] = s;
        }
        for (int j = 0; j < n; ++j) {
            const double t = -tau * work[j];
            for (int i = 0; i < m; ++i) c[i + (size_t)j * ldc] += v[(size_t)i * incv] * t;
        }
    } else {  // C := C (I - tau v v^T) ; w = C v
        for (int i = 0; i < m; ++i) work[i] = 0.0;
        for (int j = 0; j < n; ++j) {
            const double vj = v[(size_t)j * incv];
            for (int i = 0; i < m; ++i) work[i] += c[i + (size_t)j * ldc] * vj;
        }
        for (int j = 0; j < n; ++j) {
            const double t = -tau * v[(size_t)j * incv];
            for (int i = 0; i < m; ++i) c[i + (size_t)j * ldc] += work[i] * t;
        }
    }
}

void geqr2(int m, int n, double* a, int lda, double* tau, double* work) {
    const int k = std::min(m, n);
    for (int i = 0; i < k; ++i) {
        double* aii = a + i + (size_t)i * lda;
        larfg(m - i, *aii, a + std::min(i + 1, m - 1) + (size_t)i * lda, 1, tau[i]);
        if (i < n - 1) {
            const double keep = *aii;
            *aii = 1.0;
            larf('L', m - i, n - i - 1, aii, 1, tau[i], a + i + (size_t)(i + 1) * lda, lda, work);
            *aii = keep;
        }
    }
}

void orm2r(char side, char trans, int m, int n, int k, double* a, int lda, const double* tau,
           double* c, int ldc, double* work) {
    const bool left = side == 'L', notran = trans == 'N';
    const bool forward = (left && !notran) || (!left && notran);
    for (int t = 0; t < k; ++t) {
        const int i = forward ? t : k - 1 - t;
        double* aii = a + i + (size_t)i * lda;
        const double keep = *aii;
        *aii = 1.0;
        if (left) larf('L', m - i, n, aii, 1, tau[i], c + i, ldc, work);
        else larf('R', m, n - i, aii, 1, tau[i], c + (size_t)i * ldc, ldc, work);
        *aii = keep;
    }
}

// ------------------------------ ARPACK helpers ------------------------------

Which parse_which(const char* w) {
    const char a = w[0], b = w[1];
    if (a == 'L' && b == 'M') return Which::LM;
    if (a == 'S' && b == 'M') return Which::SM;
    if (a == 'L' && b == 'A') return Which::LA;
    if (a == 'S' && b == 'A') return Which::SA;
    if (a == 'B' && b == 'E') return Which::BE;
    if (a == 'L' && b == 'R') return Which::LR;
    if (a == 'S' && b == 'R') return Which::SR;
    if (a == 'L' && b == 'I') return Which::LI;
    if (a == 'S' && b == 'I') return Which::SI;
    return Which::BAD;
}

namespace {
// ARPACK's shell sort: gap n/2, n/4, ...; inner insertion walks back while
// `out_of_order(x[j], x[j+gap])`.  `swap(j, j+gap)` permutes the companions.
template <class OutOfOrder, class Swap>
void arpack_shell(int n, OutOfOrder out_of_order, Swap swap) {
    for (int gap = n / 2; gap > 0; gap /= 2)
        for (int i = gap; i <= n - 1; ++i)
            for (int j = i - gap; j >= 0 && out_of_order(j, j + gap); j -= gap) swap(j, j + gap);
}
// "out of order" predicate per `which` for the symmetric sorts (dsortr/dsesrt):
// SA -> decreasing algebraic, SM -> decreasing magnitude,
// LA -> increasing algebraic, LM -> increasing magnitude.
inline bool sym_out_of_order(Which w, double a, double b) {
    switch (w) {
        case Which::SA: return a < b;
        case Which::SM: return std::fabs(a) < std::fabs(b);
        case Which::LA: return a > b;
        case Which::LM: return std::fabs(a) > std::fabs(b);
        default: return false;
    }
}
}  // namespace

void dsortr(Which which, bool apply, int n, double* x1, double* x2) {
    if (which != Which::SA && which != Which::SM && which != Which::LA && which != Which::LM)
        return;
    arpack_shell(
        n, [&](int j, int k) { return sym_out_of_order(which, x1[j], x1[k]); },
        [&](int j, int k) {
            std::swap(x1[j], x1[k]);
            if (apply) std::swap(x2[j], x2[k]);
        });
}

void dsesrt(Which which, bool apply, int n, double* x, int na, double* a, int lda) {
    if (which != Which::SA && which != Which::SM && which != Which::LA && which != Which::LM)
        return;
    arpack_shell(
        n, [&](int j, int k) { return sym_out_of_order(which, x[j], x[k]); },
        [&](int j, int k) {
            std::swap(x[j], x[k]);
            if (apply)
                for (int i = 0; i < na; ++i) std::swap(a[i + (size_t)j * lda], a[i + (size_t)k * lda]);
        });
}

void dsgets(int ishift, Which which, int kev, int np, double* ritz, double* bounds,
            double* shifts) {
    if (which == Which::BE) {
        dsortr(Which::LA, true, kev + np, ritz, bounds);
        const int kevd2 = kev / 2;
        if (kev > 1) {
            const int cnt = std::min(kevd2, np), off = std::max(kevd2, np);
            for (int i = 0; i < cnt; ++i) {
                std::swap(ritz[i], ritz[off + i]);
                std::swap(bounds[i], bounds[off + i]);
            }
        }
    } else {
        dsortr(which, true, kev + np, ritz, bounds);
    }
    if (ishift == 1 && np > 0) {
        dsortr(Which::SM, true, np, bounds, ritz);
        std::memcpy(shifts, ritz, sizeof(double) * np);
    }
}

int dsconv(int n, const double* ritz, const double* bounds, double tol, double eps) {
    const double eps23 = std::pow(eps, 2.0 / 3.0);
    int nconv = 0;
    for (int i = 0; i < n; ++i) {
        const double temp = std::max(eps23, std::fabs(ritz[i]));
        if (bounds[i] <= tol * temp) ++nconv;
    }
    return nconv;
}

int dseigt(double rnorm, int n, const double* h, int ldh, double* eig, double* bounds,
           double* workl) {
    // eig := diag (h(:,2)); workl(1:n-1) := subdiag h(2:n,1)
    for (int i = 0; i < n; ++i) eig[i] = h[i + ldh];
    for (int i = 0; i < n - 1; ++i) workl[i] = h[i + 1];
    const int ierr = stqrb(n, eig, workl, bounds, workl + n);
    if (ierr != 0) return ierr;
    for (int k = 0; k < n; ++k) bounds[k] = rnorm * std::fabs(bounds[k]);
    return 0;
}

void dsapps_host(int kev, int np, const double* shift, double* h, int ldh, double* q, int ldq) {
    auto H1 = [&](int i) -> double& { return h[i - 1]; };         // subdiagonal column
    auto H2 = [&](int i) -> double& { return h[i - 1 + ldh]; };   // diagonal column
    auto Q = [&](int i, int j) -> double& { return q[(i - 1) + (size_t)(j - 1) * ldq]; };
    const double epsmch = kEps;
    const int kplusp = kev + np;
    for (int j = 1; j <= kplusp; ++j)
        for (int i = 1; i <= kplusp; ++i) Q(i, j) = (i == j) ? 1.0 : 0.0;
    if (np == 0) return;
    int itop = 1;
    for (int jj = 1; jj <= np; ++jj) {
        int istart = itop;
        for (;;) {  // label 20: per unreduced block
            int iend = kplusp;
            for (int i = istart; i <= kplusp - 1; ++i) {
                const double big = std::fabs(H2(i)) + std::fabs(H2(i + 1));
                if (H1(i + 1) <= epsmch * big) { H1(i + 1) = 0.0; iend = i; break; }
            }
            if (istart < iend) {
                double f = H2(istart) - shift[jj - 1];
                double g = H1(istart + 1);
                double c, s, r;
                lartg(f, g, c, s, r);
                {
                    const double a1 = c * H2(istart) + s * H1(istart + 1);
                    const double a2 = c * H1(istart + 1) + s * H2(istart + 1);
                    const double a4 = c * H2(istart + 1) - s * H1(istart + 1);
                    const double a3 = c * H1(istart + 1) - s * H2(istart);
                    H2(istart) = c * a1 + s * a2;
                    H2(istart + 1) = c * a4 - s * a3;
                    H1(istart + 1) = c * a3 + s * a4;
                }
                for (int j = 1; j <= std::min(istart + jj, kplusp); ++j) {
                    const double a1 = c * Q(j, istart) + s * Q(j, istart + 1);
                    Q(j, istart + 1) = -s * Q(j, istart) + c * Q(j, istart + 1);
                    Q(j, istart) = a1;
                }
                for (int i = istart + 1; i <= iend - 1; ++i) {
                    f = H1(i);
                    g = s * H1(i + 1);
                    H1(i + 1) = c * H1(i + 1);
                    lartg(f, g, c, s, r);
                    if (r < 0.0) { r = -r; c = -c; s = -s; }
                    H1(i) = r;
                    const double a1 = c * H2(i) + s * H1(i + 1);
                    const double a2 = c * H1(i + 1) + s * H2(i + 1);
                    const double a3 = c * H1(i + 1) - s * H2(i);
                    const double a4 = c * H2(i + 1) - s * H1(i + 1);
                    H2(i) = c * a1 + s * a2;
                    H2(i + 1) = c * a4 - s * a3;
                    H1(i + 1) = c * a3 + s * a4;
                    for (int j = 1; j <= std::min(i + jj, kplusp); ++j) {
                        const double b1 = c * Q(j, i) + s * Q(j, i + 1);
                        Q(j, i + 1) = -s * Q(j, i) + c * Q(j, i + 1);
                        Q(j, i) = b1;
                    }
                }
            }
            istart = iend + 1;
            if (H1(iend) < 0.0) {
                H1(iend) = -H1(iend);
                for (int j = 1; j <= kplusp; ++j) Q(j, iend) = -Q(j, iend);
            }
            if (iend < kplusp) continue;
            break;
        }
        for (int i = itop; i <= kplusp - 1; ++i) {
            if (H1(i + 1) > 0.0) break;
            ++itop;
        }
    }
    for (int i = itop; i <= kplusp - 1; ++i) {
        const double big = std::fabs(H2(i)) + std::fabs(H2(i + 1));
        if (H1(i + 1) <= epsmch * big) H1(i + 1) = 0.0;
    }
}

}  // namespace ahip::la
