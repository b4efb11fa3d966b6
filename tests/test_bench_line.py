"""CPU: the parts of bench.py's JSON line computed on the host.

pmc_traffic: the counter traffic a line reports must
come from a committed PMC summary of the SAME workload (operator, n, nnz,
storage, mode) -- two summaries holding the same kernel name at different n
must not be confused, and a line with no matching summary reports null with a
reason.  comm_report (VERDICT r05 missing #2): the schema of the distributed
line's per-rank collective profile."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

K_SYM = "void ahip::dev::(anonymous namespace)::k_csr_ssell<8, true, false, true>(long const*, int)"
K_DET = "void ahip::dev::(anonymous namespace)::k_csr_ssell_det<8, true, true, 6>(long const*, int)"
K_FIN = "void ahip::dev::(anonymous namespace)::k_csr_sell_fin<false, 1>(long const*, long const*)"
K_SELL = "void ahip::dev::(anonymous namespace)::k_csr_sell<4, true, true, false>(long const*)"


def _summary(path, workload, kernels):
    doc = dict(correction="x", kernels={k: dict(launches=n, traffic_bytes=b) for k, (n, b) in
                                        kernels.items()})
    if workload is not None:
        doc["workload"] = workload
    path.write_text(json.dumps(doc))


def _wl(n, nnz, storage="sym", form="sym_fixed", w="ns"):
    return dict(workload=w, n=n, nnz=nnz, storage=storage, spmv_form=form)


def test_kernel_family():
    assert bench.kernel_family(K_SYM) == "k_csr_ssell"
    assert bench.kernel_family(K_DET) == "k_csr_ssell_det"
    assert bench.kernel_family(K_FIN) == "k_csr_sell_fin"
    assert bench.kernel_family("k_vq_update(double*)") == "k_vq_update"


def test_traffic_is_keyed_by_workload(tmp_path):
    ns = _wl(10_000_000, 510_000_000)
    c2 = _wl(1_000_000, 4_996_000, w="c2")
    # the C2 summary sorts AFTER the north star's (r05w > r05s) and holds the
    # same kernel name: the round-5 line took it
    _summary(tmp_path / "r05s_pmc.json", ns, {K_SYM: (220, 2.8776e9), K_DET: (91, 2.889e9)})
    _summary(tmp_path / "r05w_c23_pmc.json", c2, {K_SYM: (351, 5.9559e7)})
    t, src, note = bench.pmc_traffic({"k_csr_ssell"}, ns, str(tmp_path))
    assert src == "r05s_pmc.json" and note is None
    assert t == 2.8776e9          # the det kernel's family is not k_csr_ssell
    t, src, _ = bench.pmc_traffic({"k_csr_ssell"}, c2, str(tmp_path))
    assert src == "r05w_c23_pmc.json" and t == 5.9559e7
    t, src, _ = bench.pmc_traffic({"k_csr_ssell"}, dict(ns, spmv_form="sym_fp64"), str(tmp_path))
    assert t is None and src is None  # that summary is the fixed-point accumulator's run


def test_traffic_null_with_reason(tmp_path):
    ns = _wl(10_000_000, 510_000_000)
    # a summary without a workload block is never used, whatever it holds
    _summary(tmp_path / "r09_pmc.json", None, {K_SYM: (10, 1.0)})
    # same workload, other storage
    _summary(tmp_path / "r08_pmc.json", _wl(10_000_000, 510_000_000, storage="full", form="full"),
             {K_FIN: (10, 5.4e9)})
    t, src, note = bench.pmc_traffic({"k_csr_ssell"}, ns, str(tmp_path))
    assert t is None and src is None
    assert "n=10000000" in note and "k_csr_ssell" in note


def test_traffic_launch_weighted_over_family(tmp_path):
    full = _wl(10_000_000, 510_000_000, storage="full", form="full")
    _summary(tmp_path / "r06_pmc.json", full, {K_FIN: (3, 10.0), K_SELL: (1, 30.0)})
    t, src, _ = bench.pmc_traffic({"k_csr_sell", "k_csr_sell_fin"}, full, str(tmp_path))
    assert src == "r06_pmc.json" and t == (3 * 10.0 + 30.0) / 4


def test_newest_matching_summary_wins(tmp_path):
    ns = _wl(10_000_000, 510_000_000)
    _summary(tmp_path / "r05s_pmc.json", ns, {K_SYM: (220, 2.0)})
    _summary(tmp_path / "r06a_pmc.json", ns, {K_SYM: (200, 3.0)})
    assert bench.pmc_traffic({"k_csr_ssell"}, ns, str(tmp_path))[:2] == (3.0, "r06a_pmc.json")


def _prof(steps, cycles, ar_ms, ar_n, h_ms, spmv_ms=10.0):
    p = {k: (0.0, 0.0, 0) for k in ("spmv", "cgs_dots", "update", "vq", "place", "finalize", "other",
                                    "allreduce", "halo")}
    p["spmv"] = (spmv_ms, 1e9, steps)
    p["update"] = (5.0, 1e9, steps)
    p["vq"] = (1.0, 1e8, cycles)
    p["allreduce"] = (ar_ms, 8.0 * 40 * ar_n, ar_n)
    p["halo"] = (h_ms, 0.0, steps)
    return p


def test_comm_report_schema():
    assert bench.comm_report(_prof(40, 2, 1.0, 80, 2.0), None, None, 0, 20.0) is None
    r = bench.comm_report(_prof(40, 2, 1.0, 80, 2.0), object(), None, 0, 20.0)
    (me,) = r["per_rank"]
    assert me["allreduce_per_step"] == 2.0 and me["halo_per_step"] == 1.0
    assert abs(me["allreduce_us_per_step"] - 25.0) < 1e-12
    assert abs(me["halo_us_per_step"] - 50.0) < 1e-12
    # kernels: spmv less its halo + update + vq
    assert abs(me["kernels_us_per_step"] - 1e3 * (10.0 - 2.0 + 5.0 + 1.0) / 40) < 1e-9
    assert abs(me["comm_ms_per_cycle"] - 1.5) < 1e-12
    assert abs(r["comm_share"] - 1.5 / 20.0) < 1e-12
    assert r["max_over_ranks"]["halo_us_per_step"] == me["halo_us_per_step"]


def test_comm_report_max_over_ranks():
    class FakeDist:
        @staticmethod
        def get_world_size():
            return 2

        @staticmethod
        def all_gather_object(out, mine):
            other = dict(mine, rank=1, halo_us_per_step=mine["halo_us_per_step"] * 3,
                         comm_ms_per_cycle=mine["comm_ms_per_cycle"] * 2)
            out[0], out[1] = mine, other

    r = bench.comm_report(_prof(40, 2, 1.0, 80, 2.0), object(), FakeDist, 0, 20.0)
    assert [x["rank"] for x in r["per_rank"]] == [0, 1]
    assert r["max_over_ranks"]["halo_us_per_step"] == 150.0
    assert abs(r["comm_share"] - 3.0 / 20.0) < 1e-12
