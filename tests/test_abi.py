"""CPU: the C-ABI library loads without a GPU and exports every entry point
include/arpack_hip.h declares (no compute calls)."""
import os
import re

from conftest import ROOT


def _declared():
    txt = open(os.path.join(ROOT, "include", "arpack_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\((?!\s*\*)", txt)) -
                  {"if", "defined", "sizeof"})


def test_header_symbols_exported(pkg):
    L = pkg.lib()
    missing = [s for s in _declared() if not hasattr(L, s)]
    assert not missing, missing


def test_reference_icb_names_covered():
    """Every ICB symbol of the implemented families is declared (ICB/arpack.h:10-21)."""
    names = _declared()
    for fam in ("ds", "dn", "zn", "ss", "sn", "cn"):  # all twelve ICB entry points
        for s in (fam + "aupd_c", fam + "eupd_c", fam + "aupd_", fam + "eupd_"):
            assert s in names, s
    for s in ("stat_c", "debug_c", "sstats_c", "sstatn_c", "cstatn_c"):
        assert s in names


def build_c_drop_in(out, ilp64=False):
    """Compile tests/c/icb_drop_in.c (a C caller written to the reference's ICB
    contract) against include/arpack_hip.h and link libarpack_hip.so, or with
    a_int = int64_t against libarpack_hip64.so (ilp64)."""
    import subprocess
    src = os.path.join(ROOT, "tests", "c", "icb_drop_in.c")
    lib = os.path.join(ROOT, "arpack-ng_amd")
    extra = ["-include", "stdint.h", "-Da_int=int64_t"] if ilp64 else []
    cmd = ["gcc", "-std=c11", "-Wall", "-Werror", "-O1", "-I", os.path.join(ROOT, "include")] + \
        extra + [src, "-L", lib, "-larpack_hip64" if ilp64 else "-larpack_hip",
                 "-Wl,-rpath," + lib, "-lm", "-o", out]
    return subprocess.run(cmd, capture_output=True, text=True)


def test_c_caller_compiles_and_links(pkg, tmp_path):
    r = build_c_drop_in(str(tmp_path / "icb_drop_in"))
    assert r.returncode == 0, r.stderr
    r = build_c_drop_in(str(tmp_path / "icb_drop_in64"), ilp64=True)
    assert r.returncode == 0, r.stderr


def test_ilp64_library_exports_reference_abi():
    """libarpack_hip64.so (a_int = int64_t) exports every reference entry point;
    the LP64 implementations it wraps are renamed ahip_lp64_* (csrc/ilp64)."""
    import ctypes
    L = ctypes.CDLL(os.path.join(ROOT, "arpack-ng_amd", "libarpack_hip64.so"))
    for fam in ("ds", "dn", "zn", "ss", "sn", "cn"):
        for s in (fam + "aupd_c", fam + "eupd_c", fam + "aupd_", fam + "eupd_"):
            assert hasattr(L, s) and hasattr(L, "ahip_lp64_" + s), s


def test_version_and_no_gpu_probe(pkg):
    assert "gfx950" in pkg.version()
    assert pkg.device_count() >= 0


def test_deterministic_env_read_at_load():
    """ARPACK_HIP_DETERMINISTIC=1 turns deterministic mode on for a fresh
    process (it was silently ignored before round 5: the library read it in a
    static initializer that left 0); arpack_hip_set_deterministic overrides it."""
    import subprocess
    import sys
    code = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); a = L.arpack_hip_deterministic(); "
            "L.arpack_hip_set_deterministic(0); print(a, L.arpack_hip_deterministic())")
    lib = os.path.join(ROOT, "arpack-ng_amd", "libarpack_hip.so")
    for val, want in (("1", "1 0"), ("0", "0 0"), (None, "0 0")):
        env = {k: v for k, v in os.environ.items() if k != "ARPACK_HIP_DETERMINISTIC"}
        if val is not None:
            env["ARPACK_HIP_DETERMINISTIC"] = val
        r = subprocess.run([sys.executable, "-c", code, lib], env=env, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.split() == want.split(), (val, r.stdout)


CPP_CALLER = r"""
#include <complex>
#include <vector>
#include "arpack.hpp"
#include "debug_c.hpp"
#include "stat_c.hpp"
template <class R> void sym() {
    a_int ido = 0, info = 0, ip[11] = {}, pt[14] = {};
    std::vector<R> r(8), v(64), w(24), l(64), d(2), z(16);
    std::vector<a_int> sel(8);
    arpack::saupd(ido, arpack::bmat::identity, 8, arpack::which::largest_algebraic, 2, R(0),
                  r.data(), 4, v.data(), 8, ip, pt, w.data(), l.data(), 48, info);
    arpack::seupd(1, arpack::howmny::ritz_vectors, sel.data(), d.data(), z.data(), 8, R(0),
                  arpack::bmat::identity, 8, arpack::which::largest_algebraic, 2, R(0), r.data(), 4,
                  v.data(), 8, ip, pt, w.data(), l.data(), 48, info);
    arpack::naupd(ido, arpack::bmat::identity, 8, arpack::which::largest_real, 2, R(0), r.data(),
                  4, v.data(), 8, ip, pt, w.data(), l.data(), 48, info);
    arpack::neupd(1, arpack::howmny::ritz_vectors, sel.data(), d.data(), d.data(), z.data(), 8,
                  R(0), R(0), w.data(), arpack::bmat::identity, 8, arpack::which::largest_real, 2,
                  R(0), r.data(), 4, v.data(), 8, ip, pt, w.data(), l.data(), 48, info);
    std::vector<std::complex<R>> c(64);
    std::vector<R> rw(4);
    arpack::naupd(ido, arpack::bmat::identity, 8, arpack::which::largest_magnitude, 2, R(0),
                  c.data(), 4, c.data(), 8, ip, pt, c.data(), c.data(), 48, rw.data(), info);
    arpack::neupd(0, arpack::howmny::ritz_vectors, sel.data(), c.data(), c.data(), 8,
                  std::complex<R>(0), c.data(), arpack::bmat::identity, 8,
                  arpack::which::largest_magnitude, 2, R(0), c.data(), 4, c.data(), 8, ip, pt,
                  c.data(), c.data(), 48, rw.data(), info);
}
int main() {
    sym<float>();
    sym<double>();
    a_int a[5];
    float t[26];
    stat_c(a[0], a[1], a[2], a[3], a[4], t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8],
           t[9], t[10], t[11], t[12], t[13], t[14], t[15], t[16], t[17], t[18], t[19], t[20], t[21],
           t[22], t[23], t[24], t[25]);
    sstatn_c();
    cstatn_c();
    debug_c(6, -6, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1);
    return 0;
}
"""


def test_cpp_caller_compiles_and_links(pkg, tmp_path):
    """A C++ caller of the reference's C++ binding (ICB/arpack.hpp, debug_c.hpp,
    stat_c.hpp; the pattern of TESTS/icb_arpack_cpp.cpp) builds unchanged
    against include/ and links libarpack_hip.so (every overload instantiated)."""
    import subprocess
    src = tmp_path / "caller.cpp"
    src.write_text(CPP_CALLER)
    lib = os.path.join(ROOT, "arpack-ng_amd")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-O1", "-I",
                        os.path.join(ROOT, "include"), str(src), "-L", lib, "-larpack_hip",
                        "-Wl,-rpath," + lib, "-o", str(tmp_path / "caller")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_stat_resets_without_gpu(pkg):
    """sstats_c / sstatn_c / cstatn_c (ICB/stat_c.h) clear the counters stat_c reads;
    no GPU call involved."""
    import ctypes
    L = pkg.lib()
    for f in ("sstats_c", "sstatn_c", "cstatn_c"):
        getattr(L, f)()
        ints = [ctypes.c_int(7) for _ in range(5)]
        flts = [ctypes.c_float(7.0) for _ in range(26)]
        L.stat_c(*[ctypes.byref(x) for x in ints + flts])
        assert [x.value for x in ints] == [0] * 5, f
        assert [x.value for x in flts] == [0.0] * 26, f
