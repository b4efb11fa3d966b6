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
    for s in ("stat_c", "debug_c", "sstats_c"):
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
