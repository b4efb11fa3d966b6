"""CPU: bench.py's multi-GPU launch plumbing.

`python bench.py --gpus N` from a plain command (no WORLD_SIZE) must start N
rank processes under torch.distributed.run before anything touches the GPU,
forward only rank 0's JSON line, and refuse N above the visible GPU count
(unless --host-transport); a rank whose WORLD_SIZE differs from --gpus must
refuse to run.  The rank side (RCCL ranks, per-rank PCI ids in the JSON line)
is exercised on the GPU box by tests/test_gpu_bench_contract.py."""
import io
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, "bench.py", *args], cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=120)


def test_more_gpus_than_visible_exits_nonzero():
    # this container has no GPU: --gpus 2 must fail loudly, not time one rank
    r = _run(["--gpus", "2"], {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "needs 2 GPUs" in r.stderr and r.stdout == ""


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"}, drop=())
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_gpus_zero_rejected():
    r = _run(["--gpus", "0"])
    assert r.returncode == 2


class _FakeProc:
    def __init__(self, cmd, **kw):
        _FakeProc.last = (cmd, kw)
        self.stdout = io.StringIO(
            "[Gloo] Rank 0 is connected to 1 peer ranks.\n"
            '{"metric": "m", "value": 1.0, "n_gpus": 4}\n'
            '{"not": "the bench line"}\n'
            "RCCL version 2.x\n")

    def wait(self):
        return 0

    def send_signal(self, s):
        pass


def test_launcher_command_and_forwarding(monkeypatch, capsys):
    monkeypatch.setattr(bench.subprocess, "Popen", _FakeProc)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 8)
    args = bench.argparse.Namespace(gpus=4, host_transport=False)
    argv = ["--gpus", "4", "--steps", "3", "--warmup", "1"]
    rc = bench.launch_ranks(args, argv)
    assert rc == 0
    cmd, kw = _FakeProc.last
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(c.startswith("--master-port=") for c in cmd)
    assert cmd[-len(argv):] == argv and cmd[-len(argv) - 1].endswith("bench.py")
    assert kw["env"]["MASTER_ADDR"] == "127.0.0.1"
    out, err = capsys.readouterr()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    assert lines == ['{"metric": "m", "value": 1.0, "n_gpus": 4}']
    assert "Gloo" in err and "RCCL version" in err and "not" in err


def test_launcher_refuses_without_gpus(monkeypatch, capsys):
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    called = []
    monkeypatch.setattr(bench.subprocess, "Popen", lambda *a, **k: called.append(a))
    rc = bench.launch_ranks(bench.argparse.Namespace(gpus=2, host_transport=False), ["--gpus", "2"])
    assert rc == 2 and not called
    # a rehearsal on one GPU is allowed
    monkeypatch.setattr(bench.subprocess, "Popen", _FakeProc)
    rc = bench.launch_ranks(bench.argparse.Namespace(gpus=2, host_transport=True),
                            ["--gpus", "2", "--host-transport"])
    assert rc == 0


def test_launcher_without_json_line_fails(monkeypatch):
    class Quiet(_FakeProc):
        def __init__(self, cmd, **kw):
            super().__init__(cmd, **kw)
            self.stdout = io.StringIO("nothing\n")
    monkeypatch.setattr(bench.subprocess, "Popen", Quiet)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 8)
    assert bench.launch_ranks(bench.argparse.Namespace(gpus=2, host_transport=False), []) == 1
