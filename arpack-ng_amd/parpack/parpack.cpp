// libparpack_hip.so -- PARPACK's drop-in boundary over the MI355X engine.
//
// Exports exactly the entry points a PARPACK caller binds:
//   * the ISO_C_BINDING layer, ICB/parpack.h:17-33 (implemented in the
//     reference by PARPACK/SRC/MPI/icbp[sdcz][sn].F90): p[sd]saupd_c,
//     p[sd]seupd_c, p[sd]naupd_c, p[sd]neupd_c, p[cz]naupd_c, p[cz]neupd_c,
//     each taking the Fortran handle of an MPI communicator (MPI_Fint) and n =
//     this process's rows;
//   * the Fortran symbols p[sd]saupd_ ... p[cz]neupd_ (PARPACK/SRC/MPI/pdsaupd.f:
//     `subroutine pdsaupd(comm, ido, bmat, n, ...)`: every argument by
//     reference, hidden trailing CHARACTER lengths), so the reference's own
//     Fortran drivers (PARPACK/EXAMPLES/MPI/*.f) link unchanged.
//
// Each call maps the caller's communicator onto the engine's (one process per
// rank): a row decomposition of the local sizes (MPI_Exscan / MPI_Allreduce,
// the caller's rows in rank order, as PARPACK assumes), PARPACK's per-rank
// start vector (PARPACK/SRC/MPI/pdgetv0.f:234-245), and the transport of the
// engine's reductions:
//   * RCCL when every rank on a node has a GPU of its own (the 128-byte unique
//     id broadcast over MPI; device = the rank's index on its node);
//   * otherwise (several ranks sharing a GPU, ARPACK_HIP_PCOMM=host) the
//     engine's host-staged transport with MPI_Allreduce on a private duplicate
//     of the caller's communicator.
// The solve itself -- Arnoldi/Lanczos steps, reductions, restarts, V*Q -- is
// the engine's (libarpack_hip.so, arpack_hip_p*aupd_c); V, resid and workd stay
// where the caller put them (host arrays are mirrored in HBM).
#include <mpi.h>

#include <cfloat>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <utility>
#include <vector>

#include "../../include/arpack_hip.h"

namespace {

struct Binding {
    MPI_Fint key = 0;             // the caller's communicator (Fortran handle)
    MPI_Comm comm = MPI_COMM_NULL;  // private duplicate for the engine's collectives
    int rank = 0, size = 1;
    bool rccl = false;
};

std::mutex g_mu;
Binding g_bind;
bool g_bound = false;
// one decomposition per (communicator, local rows, first row, global rows);
// they stay alive for the *eupd call that follows the *aupd loop (and for
// later solves).  g_cur: the decomposition of the solve in progress on a
// (communicator, local rows) pair, fixed at its ido = 0 call.
using DistKey = std::tuple<MPI_Fint, int64_t, long long, long long>;
std::map<DistKey, arpack_hip_dist*> g_dists;
std::map<std::pair<MPI_Fint, int64_t>, arpack_hip_dist*> g_cur;

void host_allreduce(double* buf, int count, void* ctx) {
    MPI_Allreduce(MPI_IN_PLACE, buf, count, MPI_DOUBLE, MPI_SUM, static_cast<Binding*>(ctx)->comm);
}

// one group of the engine's point-to-point transfers (arpack_hip.h's host
// p2p contract): every transfer posted non-blocking, then all completed; one
// tag, so transfers between a pair match in posting order
void host_p2p(int nops, const int* peer, const int* is_send, double* const* buf,
              const int64_t* count, void* ctx) {
    auto* b = static_cast<Binding*>(ctx);
    std::vector<MPI_Request> rq((size_t)nops);
    for (int k = 0; k < nops; ++k) {
        if (is_send[k]) MPI_Isend(buf[k], (int)count[k], MPI_DOUBLE, peer[k], 71, b->comm, &rq[k]);
        else MPI_Irecv(buf[k], (int)count[k], MPI_DOUBLE, peer[k], 71, b->comm, &rq[k]);
    }
    if (nops) MPI_Waitall(nops, rq.data(), MPI_STATUSES_IGNORE);
}

void release_binding() {
    for (auto& kv : g_dists) arpack_hip_dist_destroy(kv.second);
    g_dists.clear();
    g_cur.clear();
    if (g_bound) {
        arpack_hip_comm_destroy();
        int fin = 0;
        MPI_Finalized(&fin);
        if (!fin && g_bind.comm != MPI_COMM_NULL) MPI_Comm_free(&g_bind.comm);
    }
    g_bind = Binding{};
    g_bound = false;
}

// V arrays of the solves in progress (from a fresh *aupd call to its ido = 99
// return): the engine keeps their state next to the communicator binding.
std::set<const void*> g_live;
void live_begin(const void* v, const a_int* ido) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (*ido == 0) g_live.erase(v);  // a new solve on V abandons the old one
}
void live_end(const void* v, const a_int* ido) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (*ido == 99) g_live.erase(v);
    else g_live.insert(v);
}

// Bind the engine's communicator to `fcomm` (collective over it on first use;
// the caller holds g_mu).  One communicator at a time: a continuing call or an
// *eupd on another communicator while a solve is in progress is refused
// (info = -9999) rather than freeing that solve's distribution under it.  A
// fresh *aupd (ido = 0) on another communicator starts a new solve and
// abandons the ones in progress, as a fresh call abandons the previous solve
// in the reference (one SAVEd state per routine): their later calls on the old
// communicator find no binding and return -9999, so an abandoned solve cannot
// block rebinding for the rest of the process.
bool bind_comm(MPI_Fint fcomm, bool fresh) {
    if (g_bound && g_bind.key == fcomm) return true;
    if (g_bound && !g_live.empty() && !fresh) return false;
    g_live.clear();
    release_binding();
    MPI_Comm c = MPI_Comm_f2c(fcomm);
    Binding b;
    b.key = fcomm;
    if (MPI_Comm_dup(c, &b.comm) != MPI_SUCCESS) return false;
    MPI_Comm_rank(b.comm, &b.rank);
    MPI_Comm_size(b.comm, &b.size);
    // ranks on this node and my index among them
    MPI_Comm node;
    MPI_Comm_split_type(b.comm, MPI_COMM_TYPE_SHARED, b.rank, MPI_INFO_NULL, &node);
    int lrank = 0, lsize = 1;
    MPI_Comm_rank(node, &lrank);
    MPI_Comm_size(node, &lsize);
    MPI_Comm_free(&node);
    const char* mode = std::getenv("ARPACK_HIP_PCOMM");
    const int ndev = arpack_hip_device_count();
    int want_rccl = ndev >= lsize && !(mode && std::strcmp(mode, "host") == 0) ? 1 : 0;
    int all_rccl = 0;  // every rank must agree on the transport
    MPI_Allreduce(&want_rccl, &all_rccl, 1, MPI_INT, MPI_MIN, b.comm);
    b.rccl = all_rccl != 0;
    g_bind = b;
    int rc = 0;
    if (b.rccl) {
        // rank 0's RCCL id and whether it got one, in one broadcast: on failure
        // no rank enters the RCCL bootstrap (which would wait for rank 0)
        char id[129] = {0};
        if (b.rank == 0 && arpack_hip_comm_unique_id(id) != 0) id[128] = 1;
        MPI_Bcast(id, 129, MPI_CHAR, 0, b.comm);
        rc = id[128] ? -1 : arpack_hip_comm_init(b.size, b.rank, id, lrank);
    } else {
        rc = arpack_hip_comm_init_host(b.size, b.rank, host_allreduce, host_p2p, &g_bind,
                                       ndev > 0 ? lrank % ndev : 0);
    }
    int ok = rc == 0 ? 1 : 0, all = 0;
    MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, b.comm);
    if (!all) {
        if (rc == 0) arpack_hip_comm_destroy();
        MPI_Comm_free(&g_bind.comm);
        g_bind = Binding{};
        return false;
    }
    g_bound = true;
    return true;
}

// The decomposition of this call: nloc local rows, row0 = rows of the lower
// ranks, n_global = all rows.  At a solve's first call (fresh: *aupd with ido =
// 0) it is established collectively -- MPI_Exscan / MPI_Allreduce of the local
// sizes, then an agreement that every rank has its decomposition, so a rank
// whose setup fails never leaves the others waiting in the solve's collectives
// (all of them return info = -9999) -- and it serves the later calls of the
// same solve and the *eupd call after it (no collective per RCI call).
arpack_hip_dist* dist_for(MPI_Fint fcomm, int64_t nloc, bool fresh) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (!bind_comm(fcomm, fresh)) return nullptr;
    const auto cur = std::make_pair(fcomm, nloc);
    if (!fresh) {
        auto it = g_cur.find(cur);
        if (it != g_cur.end()) return it->second;
    }
    long long mine = nloc, row0 = 0, nglob = 0;
    MPI_Exscan(&mine, &row0, 1, MPI_LONG_LONG, MPI_SUM, g_bind.comm);
    if (g_bind.rank == 0) row0 = 0;  // MPI_Exscan leaves rank 0's result undefined
    MPI_Allreduce(&mine, &nglob, 1, MPI_LONG_LONG, MPI_SUM, g_bind.comm);
    const DistKey key{fcomm, nloc, row0, nglob};
    arpack_hip_dist* D = nullptr;
    auto it = g_dists.find(key);
    if (it != g_dists.end()) {
        D = it->second;
    } else if (nloc > 0 && arpack_hip_dist_rows(&D, nloc, row0, nglob) == 0) {
        arpack_hip_dist_set_seed_mode(D, 1);  // PARPACK's per-rank start vector
        g_dists[key] = D;
    } else {
        D = nullptr;
    }
    int ok = D ? 1 : 0, all = 0;
    MPI_Allreduce(&ok, &all, 1, MPI_INT, MPI_MIN, g_bind.comm);
    if (!all) {
        g_cur.erase(cur);
        return nullptr;
    }
    g_cur[cur] = D;
    return D;
}

void fail(a_int* ido, a_int* info) {  // no decomposition (MPI / device setup failed)
    *info = -9999;
    if (ido) *ido = 99;
}

// LAPACK's scaled 2-norm (dnrm2 / dznrm2 without overflow), local part
template <class T>
double nrm2_local(a_int n, const T* x, a_int inc, int comps) {
    double scale = 0.0, ssq = 1.0;
    for (a_int i = 0; i < n; ++i)
        for (int c = 0; c < comps; ++c) {
            const double v = (double)x[(int64_t)i * inc * comps + c];
            if (v != 0.0) {
                const double a = v < 0 ? -v : v;
                if (scale < a) {
                    ssq = 1.0 + ssq * (scale / a) * (scale / a);
                    scale = a;
                } else {
                    ssq += (a / scale) * (a / scale);
                }
            }
        }
    return scale * std::sqrt(ssq);
}

// p?norm2 (PARPACK/SRC/MPI/pdnorm2.f): the local norm, the MAX over the ranks,
// then max * sqrt(SUM (local/max)^2) -- overflow-safe, as the reference does
template <class T>
double pnorm2(MPI_Fint fcomm, a_int n, const T* x, a_int inc, int comps) {
    MPI_Comm c = MPI_Comm_f2c(fcomm);
    const double loc = nrm2_local(n, x, inc, comps);
    double mx = 0.0;
    MPI_Allreduce(&loc, &mx, 1, MPI_DOUBLE, MPI_MAX, c);
    if (mx == 0.0) return 0.0;
    const double b = (loc / mx) * (loc / mx);
    double s = 0.0;
    MPI_Allreduce(&b, &s, 1, MPI_DOUBLE, MPI_SUM, c);
    return mx * std::sqrt(s < 0 ? -s : s);
}

// Fortran tol (by reference): tol <= 0 becomes eps in the caller's variable at
// ido = 0 (SRC/dsaupd.f:550 / pdsaupd.f), which the by-value C entry cannot do
template <class T>
void fortran_tol(const a_int* ido, T* tol) {
    if (*ido == 0 && *tol <= T(0)) *tol = std::is_same_v<T, double> ? DBL_EPSILON * 0.5 : FLT_EPSILON * 0.5f;
}

using zc = a_dcomplex;
using cc = a_fcomplex;

}  // namespace

extern "C" {

// ---- ISO_C_BINDING layer (ICB/parpack.h) -------------------------------------
void pdsaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
               a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_pdsaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, info);
    live_end(v, ido);
}
void pdseupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, double* d,
               double* z, a_int ldz, double sigma, char const* bmat, a_int n, char const* which,
               a_int nev, double tol, double* resid, a_int ncv, double* v, a_int ldv,
               a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int lworkl,
               a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_pdseupd_c(D, rvec, howmny, select, d, z, ldz, sigma, bmat, n, which, nev, tol,
                         resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl, info);
}
void pssaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
               a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_pssaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, info);
    live_end(v, ido);
}
void psseupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, float* d,
               float* z, a_int ldz, float sigma, char const* bmat, a_int n, char const* which,
               a_int nev, float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
               a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_psseupd_c(D, rvec, howmny, select, d, z, ldz, sigma, bmat, n, which, nev, tol,
                         resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl, info);
}
void pdnaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               double tol, double* resid, a_int ncv, double* v, a_int ldv, a_int* iparam,
               a_int* ipntr, double* workd, double* workl, a_int lworkl, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_pdnaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, info);
    live_end(v, ido);
}
void pdneupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, double* dr,
               double* di, double* z, a_int ldz, double sigmar, double sigmai, double* workev,
               char const* bmat, a_int n, char const* which, a_int nev, double tol, double* resid,
               a_int ncv, double* v, a_int ldv, a_int* iparam, a_int* ipntr, double* workd,
               double* workl, a_int lworkl, a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_pdneupd_c(D, rvec, howmny, select, dr, di, z, ldz, sigmar, sigmai, workev, bmat, n,
                         which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
                         info);
}
void psnaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               float tol, float* resid, a_int ncv, float* v, a_int ldv, a_int* iparam,
               a_int* ipntr, float* workd, float* workl, a_int lworkl, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_psnaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, info);
    live_end(v, ido);
}
void psneupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, float* dr,
               float* di, float* z, a_int ldz, float sigmar, float sigmai, float* workev,
               char const* bmat, a_int n, char const* which, a_int nev, float tol, float* resid,
               a_int ncv, float* v, a_int ldv, a_int* iparam, a_int* ipntr, float* workd,
               float* workl, a_int lworkl, a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_psneupd_c(D, rvec, howmny, select, dr, di, z, ldz, sigmar, sigmai, workev, bmat, n,
                         which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl,
                         info);
}
void pznaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               double tol, zc* resid, a_int ncv, zc* v, a_int ldv, a_int* iparam, a_int* ipntr,
               zc* workd, zc* workl, a_int lworkl, double* rwork, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_pznaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, rwork, info);
    live_end(v, ido);
}
void pzneupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, zc* d, zc* z,
               a_int ldz, zc sigma, zc* workev, char const* bmat, a_int n, char const* which,
               a_int nev, double tol, zc* resid, a_int ncv, zc* v, a_int ldv, a_int* iparam,
               a_int* ipntr, zc* workd, zc* workl, a_int lworkl, double* rwork, a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_pzneupd_c(D, rvec, howmny, select, d, z, ldz, sigma, workev, bmat, n, which, nev, tol,
                         resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl, rwork, info);
}
void pcnaupd_c(MPI_Fint comm, a_int* ido, char const* bmat, a_int n, char const* which, a_int nev,
               float tol, cc* resid, a_int ncv, cc* v, a_int ldv, a_int* iparam, a_int* ipntr,
               cc* workd, cc* workl, a_int lworkl, float* rwork, a_int* info) {
    live_begin(v, ido);
    arpack_hip_dist* D = dist_for(comm, n, *ido == 0);
    if (!D) return fail(ido, info);
    arpack_hip_pcnaupd_c(D, ido, bmat, n, which, nev, tol, resid, ncv, v, ldv, iparam, ipntr, workd,
                         workl, lworkl, rwork, info);
    live_end(v, ido);
}
void pcneupd_c(MPI_Fint comm, a_int rvec, char const* howmny, a_int const* select, cc* d, cc* z,
               a_int ldz, cc sigma, cc* workev, char const* bmat, a_int n, char const* which,
               a_int nev, float tol, cc* resid, a_int ncv, cc* v, a_int ldv, a_int* iparam,
               a_int* ipntr, cc* workd, cc* workl, a_int lworkl, float* rwork, a_int* info) {
    arpack_hip_dist* D = dist_for(comm, n, false);
    if (!D) return fail(nullptr, info);
    arpack_hip_pcneupd_c(D, rvec, howmny, select, d, z, ldz, sigma, workev, bmat, n, which, nev, tol,
                         resid, ncv, v, ldv, iparam, ipntr, workd, workl, lworkl, rwork, info);
}

// ---- Fortran symbols (PARPACK/SRC/MPI/p*aupd.f, p*eupd.f): by reference +
//      hidden CHARACTER lengths; LOGICAL rvec / select as 4-byte integers ----
void pdsaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, double* tol, double* resid, a_int* ncv, double* v, a_int* ldv,
              a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int* lworkl,
              a_int* info, size_t, size_t) {
    fortran_tol(ido, tol);
    pdsaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, info);
}
void pdseupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, double* d,
              double* z, a_int* ldz, double* sigma, char const* bmat, a_int* n, char const* which,
              a_int* nev, double* tol, double* resid, a_int* ncv, double* v, a_int* ldv,
              a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int* lworkl,
              a_int* info, size_t, size_t, size_t) {
    pdseupd_c(*comm, *rvec, howmny, select, d, z, *ldz, *sigma, bmat, *n, which, *nev, *tol, resid,
              *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, info);
}
void pssaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, float* tol, float* resid, a_int* ncv, float* v, a_int* ldv,
              a_int* iparam, a_int* ipntr, float* workd, float* workl, a_int* lworkl, a_int* info,
              size_t, size_t) {
    fortran_tol(ido, tol);
    pssaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, info);
}
void psseupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, float* d, float* z,
              a_int* ldz, float* sigma, char const* bmat, a_int* n, char const* which, a_int* nev,
              float* tol, float* resid, a_int* ncv, float* v, a_int* ldv, a_int* iparam,
              a_int* ipntr, float* workd, float* workl, a_int* lworkl, a_int* info, size_t, size_t,
              size_t) {
    psseupd_c(*comm, *rvec, howmny, select, d, z, *ldz, *sigma, bmat, *n, which, *nev, *tol, resid,
              *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, info);
}
void pdnaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, double* tol, double* resid, a_int* ncv, double* v, a_int* ldv,
              a_int* iparam, a_int* ipntr, double* workd, double* workl, a_int* lworkl,
              a_int* info, size_t, size_t) {
    fortran_tol(ido, tol);
    pdnaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, info);
}
void pdneupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, double* dr,
              double* di, double* z, a_int* ldz, double* sigmar, double* sigmai, double* workev,
              char const* bmat, a_int* n, char const* which, a_int* nev, double* tol,
              double* resid, a_int* ncv, double* v, a_int* ldv, a_int* iparam, a_int* ipntr,
              double* workd, double* workl, a_int* lworkl, a_int* info, size_t, size_t, size_t) {
    pdneupd_c(*comm, *rvec, howmny, select, dr, di, z, *ldz, *sigmar, *sigmai, workev, bmat, *n,
              which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, info);
}
void psnaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, float* tol, float* resid, a_int* ncv, float* v, a_int* ldv,
              a_int* iparam, a_int* ipntr, float* workd, float* workl, a_int* lworkl, a_int* info,
              size_t, size_t) {
    fortran_tol(ido, tol);
    psnaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, info);
}
void psneupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, float* dr,
              float* di, float* z, a_int* ldz, float* sigmar, float* sigmai, float* workev,
              char const* bmat, a_int* n, char const* which, a_int* nev, float* tol, float* resid,
              a_int* ncv, float* v, a_int* ldv, a_int* iparam, a_int* ipntr, float* workd,
              float* workl, a_int* lworkl, a_int* info, size_t, size_t, size_t) {
    psneupd_c(*comm, *rvec, howmny, select, dr, di, z, *ldz, *sigmar, *sigmai, workev, bmat, *n,
              which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, info);
}
void pznaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, double* tol, zc* resid, a_int* ncv, zc* v, a_int* ldv, a_int* iparam,
              a_int* ipntr, zc* workd, zc* workl, a_int* lworkl, double* rwork, a_int* info,
              size_t, size_t) {
    fortran_tol(ido, tol);
    pznaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, rwork, info);
}
void pzneupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, zc* d, zc* z,
              a_int* ldz, zc* sigma, zc* workev, char const* bmat, a_int* n, char const* which,
              a_int* nev, double* tol, zc* resid, a_int* ncv, zc* v, a_int* ldv, a_int* iparam,
              a_int* ipntr, zc* workd, zc* workl, a_int* lworkl, double* rwork, a_int* info, size_t,
              size_t, size_t) {
    pzneupd_c(*comm, *rvec, howmny, select, d, z, *ldz, *sigma, workev, bmat, *n, which, *nev, *tol,
              resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, rwork, info);
}
void pcnaupd_(MPI_Fint* comm, a_int* ido, char const* bmat, a_int* n, char const* which,
              a_int* nev, float* tol, cc* resid, a_int* ncv, cc* v, a_int* ldv, a_int* iparam,
              a_int* ipntr, cc* workd, cc* workl, a_int* lworkl, float* rwork, a_int* info, size_t,
              size_t) {
    fortran_tol(ido, tol);
    pcnaupd_c(*comm, ido, bmat, *n, which, *nev, *tol, resid, *ncv, v, *ldv, iparam, ipntr, workd,
              workl, *lworkl, rwork, info);
}
void pcneupd_(MPI_Fint* comm, a_int* rvec, char const* howmny, a_int* select, cc* d, cc* z,
              a_int* ldz, cc* sigma, cc* workev, char const* bmat, a_int* n, char const* which,
              a_int* nev, float* tol, cc* resid, a_int* ncv, cc* v, a_int* ldv, a_int* iparam,
              a_int* ipntr, cc* workd, cc* workl, a_int* lworkl, float* rwork, a_int* info, size_t,
              size_t, size_t) {
    pcneupd_c(*comm, *rvec, howmny, select, d, z, *ldz, *sigma, workev, bmat, *n, which, *nev, *tol,
              resid, *ncv, v, *ldv, iparam, ipntr, workd, workl, *lworkl, rwork, info);
}

// ---- PARPACK's collective norms (PARPACK/SRC/MPI/pdnorm2.f, pdznorm2.f,
//      psnorm2.f, pscnorm2.f), which the reference's drivers call directly ----
double pdnorm2_(MPI_Fint* comm, a_int* n, const double* x, a_int* inc) {
    return pnorm2(*comm, *n, x, *inc, 1);
}
double pdznorm2_(MPI_Fint* comm, a_int* n, const double* x, a_int* inc) {
    return pnorm2(*comm, *n, x, *inc, 2);
}
float psnorm2_(MPI_Fint* comm, a_int* n, const float* x, a_int* inc) {
    return (float)pnorm2(*comm, *n, x, *inc, 1);
}
float pscnorm2_(MPI_Fint* comm, a_int* n, const float* x, a_int* inc) {
    return (float)pnorm2(*comm, *n, x, *inc, 2);
}

}  // extern "C"
