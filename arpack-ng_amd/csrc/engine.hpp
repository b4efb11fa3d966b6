// Engine internals shared by the symmetric solver, the post-processing and the
// C-ABI layer.
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <memory>
#include <optional>
#include <vector>

#include "dense.hpp"
#include "device.hpp"
#include "dist.hpp"
#include "dgen.hpp"
#include "dshift.hpp"
#include "rci.hpp"

namespace ahip {

// /timing/ common-block counters (stat.h:8-21); the timers of the reference
// are dead in its default build (UTIL/second_NONE.f:31) and are reported as 0.
struct Stats {
    int nopx = 0, nbx = 0, nrorth = 0, nitref = 0, nrstrt = 0;
};
extern Stats g_stats;

// The process-wide SAVEd LAPACK seed of each start-vector routine, kept as the
// 48-bit integer its four base-4096 digits encode: dgetv0 (shared by dsaupd and
// dnaupd), sgetv0, zgetv0 and cgetv0 each keep their own, initialised to
// (1,3,5,7) on first use (SRC/dgetv0.f:202-208, sgetv0.f, zgetv0.f, cgetv0.f).
// family: 'd', 's', 'z', 'c'.
uint64_t& getv0_seed(char family);
// PARPACK's p?getv0 seed (PARPACK/SRC/MPI/pdgetv0.f:225-246): per process rank,
// the digits of 1000 + 2 rank + 1, SAVEd per family like the serial one.
uint64_t& pgetv0_seed(char family, int rank);
uint64_t seed48_from_iseed(const int iseed[4]);
void iseed_from_seed48(uint64_t s, int iseed[4]);
uint64_t lcg_advance(uint64_t seed, uint64_t steps);  // seed * a^steps mod 2^48

// Caller-visible arrays in one place. `dev_*` are what the kernels use: the
// caller's own buffers in device-pointer mode, engine-owned mirrors in
// host-pointer mode.  R is the storage type (double: d*, float: s*).
template <class R>
struct ArraysT {
    bool host_mode = true;
    int64_t n = 0;
    int ncv = 0;
    R* h_resid = nullptr;
    R* h_v = nullptr;
    int h_ldv = 0;
    R* h_workd = nullptr;
    R* d_resid = nullptr;
    R* d_v = nullptr;
    int64_t d_ld = 0;
    R* d_workd = nullptr;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    DevErr err;  // first failed HIP call of this solve (sticky)
    dev::FinQueue* defq = nullptr;  // the solve's deferred finalize, launched by sync()
    void ck(hipError_t e) { err.ck(e); }

    // fails with a negative code if pointer kinds are mixed
    int attach(int64_t n, int ncv, R* resid, R* v, int ldv, R* workd);
    void release();
    void upload_resid();
    void download_all();           // V, resid, workd -> caller (host mode)
    void d2h_workd(int64_t off, int64_t len);
    void h2d_workd(int64_t off, int64_t len);
    void sync();
};
using Arrays = ArraysT<double>;

// dlamch / slamch constants of a family (SRC/dsaupd.f:550, SRC/ssaupd.f:550)
template <class R>
struct Prec;
template <>
struct Prec<double> {
    static constexpr double eps = DBL_EPSILON * 0.5;  // dlamch('E')
    static constexpr double safmin = DBL_MIN;         // dlamch('S')
};
template <>
struct Prec<float> {
    static constexpr double eps = FLT_EPSILON * 0.5;  // slamch('E')
    static constexpr double safmin = FLT_MIN;         // slamch('S')
};

bool is_device_pointer(const void* p);
hipStream_t default_stream();  // set through arpack_hip_set_stream()

// One implicitly restarted Krylov solve: symmetric Lanczos (dsaupd family,
// sym.cpp) or nonsymmetric Arnoldi (dnaupd family, ns.cpp).  The n-length
// step machinery (getv0, the Lanczos/Arnoldi step with CGS + DGKS, V*Q) is
// shared; only the ncv-sized host work differs.  R is the storage type of the
// n-length data (double: dsaupd/dnaupd, float: ssaupd/snaupd); the ncv-sized
// host work is done in double in both (workl is a double shadow for float).
template <class R>
class SolverT {
public:
    // configuration fixed at ido == 0 (SRC/dsaupd.f:473-596)
    char bmat = 'I';
    la::Which which = la::Which::LM;
    int n = 0, ncv = 0, mode = 1, ishift = 1, mxiter = 0;
    int nev0 = 0, np = 0;     // dsaupd's nev0 / np (updated by the loop)
    int lworkl = 0;
    // per-call
    double tol = 0.0;
    int* iparam = nullptr;
    int* ipntr = nullptr;
    double* workl = nullptr;   // host view of the caller's workl
    int info = 0;

    ArraysT<R> a;
    dev::Workspace ws;
    RciCtx ctx;
    std::optional<Task> root;

    // free-running mode (arpack_hip_dsaupd_csr): OP requests are served by
    // an on-device CSR operator without returning to the caller.
    bool free_run = false;
    // cycle-granular pausing of the free-running driver (bench timing): at the
    // top of each restart cycle, if pause_budget == 0 the solve parks with
    // ido = kPauseIdo; -1 disables.
    static constexpr int kPauseIdo = 98;
    int pause_budget = -1;
    // multi-GPU row-block distribution (nullptr: single GPU): n is then the
    // LOCAL row count and row0 the global index of local row 0
    const DistOp* dist = nullptr;
    uint64_t dist_gen = 0;  // generation of dist->comm when the solve started
    int64_t row0 = 0;
    const dev::Csr* csr = nullptr;
    // mode 3 free run (arpack_hip_dsaupd_shift): OP = (A - sigma I)^{-1} by the
    // device CG of dshift.hip on csr = shift->A
    dev::DShift* shift = nullptr;
    // generalized modes free run (arpack_hip_dsaupd_gen): OP*x and B*x on the
    // device (csr = gen->A)
    dev::DGen* gen = nullptr;

    // nonsymmetric Arnoldi (dnaupd): full upper-Hessenberg H (ld ncv)
    bool arnoldi = false;
    int64_t n_global = 0;  // problem dimension (enters dnaitr/dnapps' smlnum)
    // workl offsets (0-based) of h, ritz (ritzr), ritzi, bounds, q, w
    int ih = 0, iritz = 0, iritzi = 0, ibounds = 0, iq = 0, iw = 0;
    double rnorm = 0.0;  // host copy of dsaup2's rnorm
    bool rnorm_stale = false;  // rnorm lives only on the device until the next cycle ends
    std::vector<double> hcol_h;  // Arnoldi: the cycle's new H columns, downloaded with the state
    R* ybuf = nullptr;  // free-running: OP's y on 128-B lines when workd(irj) is not (saitr)
    // machine constants of the family (convergence tests, tol <= 0 default)
    double eps = Prec<R>::eps, safmin = Prec<R>::safmin;
    // float family: the double shadow of the caller's workl (workl points here)
    std::vector<double> wshadow;

    ~SolverT();
    Task run();     // dsaup2
    Task run_ns();  // dnaup2

    // A failed HIP call of this solve (a.err) ends it with info = -9999.  On a
    // row distribution the ranks first agree (one flag allreduce, at points
    // every rank reaches in the same order: once per restart cycle), so they
    // leave the restart loop together; `halted` holds the agreed verdict.
    bool halted = false;
    bool check_halt();

private:
    Task getv0(bool initv, int j, int itry, int& ierr);
    Task saitr(int k, int npk, int& iinfo);
    void sapps(int kev, int npk);
    void vq_device(int kev, int kplusp, double sigmak, double betak);
    RciAwait rci(int ido, int64_t x, int64_t y, int64_t bx = -1);
    RciAwait op(int ido, int64_t x, int64_t y, int64_t bx, const R* xp, R* yp);
    void read_state();
    void write_state();
    void fin(int m, dev::FinPhase ph, int j, int rstart, int gate, int m2 = 0, int rstart_prev = 0,
             bool defer = false);
    R* vcol(int j) { return a.d_v + (int64_t)(j - 1) * a.d_ld; }  // 1-based column
    R* dist_x();  // the distributed operator's x window (double only)
    void dgks2_tail(int j, int rstart);
public:
    const R* op_x = nullptr;  // device pointers of the pending OP request
    R* op_y = nullptr;
    // overlapped distributed SpMV (RCCL, > 1 rank): the folded update pass
    // records x_ev once the SpMV's input is written; the driver runs the halo +
    // SpMV on op_stream after it, concurrently with the update's allreduce and
    // finalize on a.stream, and a.stream waits y_ev before the next pass
    hipStream_t op_stream = nullptr;
    hipEvent_t x_ev = nullptr, y_ev = nullptr;
    bool x_ready = false;
    bool overlap_ready();  // creates the stream/events on first use
};
using Solver = SolverT<double>;

}  // namespace ahip
