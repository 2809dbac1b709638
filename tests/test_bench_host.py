"""bench.py's host logic without a GPU: the multi-rank exchange check's failure reporting (a
rank whose communicator cannot be built reports the error on the line instead of raising, and
the ranks still meet at the closing all-reduce), and the argument surface the driver uses."""
import importlib.util
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_host", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


class _FakeCtx:
    closed = False

    def __init__(self, *a, **kw):
        pass

    def close(self):
        _FakeCtx.closed = True


class _FakeKnn:
    Context = _FakeCtx

    @staticmethod
    def comm_unique_id():
        return b"\0" * 128

    class Comm:
        def __init__(self, *a, **kw):
            raise RuntimeError("knn_comm_create: RCCL unavailable")


def test_exchange_check_reports_errors():
    import torch
    import torch.distributed as dist
    b = _bench()
    out = b.rccl_exchange_check(_FakeKnn, torch, dist, 0, 1, 0, True, 1)
    assert out["status"] == "error" and "RCCL unavailable" in out["error"]
    assert out["equal_to_whole_train_path"] is False
    assert out["ranks"] == 1 and _FakeCtx.closed


def test_bench_flags():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0
    for flag in ("--gpus", "--steps", "--warmup", "--config", "--shard", "--strong", "--data", "--no-bit-match"):
        assert flag in r.stdout


def test_default_scaling_is_strong():
    """The --gpus N line times BASELINE's fixed problem by default (weak scaling
    only behind --weak)."""
    b = _bench()
    for cfg in ("A", "B", "C", "C1"):
        assert b.CONFIGS[cfg][6] == "strong", cfg
        assert b.resolve_scaling(b.CONFIGS[cfg][8]) == "strong"
    assert b.resolve_scaling("test", weak=True) == "weak"
    assert b.resolve_scaling("train", weak=True) == "strong"  # train-sharded: always the fixed set
    import pytest
    with pytest.raises(SystemExit):
        b.resolve_scaling("test", strong=True, weak=True)


def test_watchdog_timeout_exits_nonzero():
    """A hung exchange check ends the run with a non-zero status and the line still printed
    (it used to exit 0, hiding the hang inside the JSON)."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench.run_with_watchdog(lambda: time.sleep(30), 0.5, {'metric': 'x'}, 0); print('not reached')"
            % REPO)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 3, (r.returncode, r.stderr[-500:])
    import json
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["rccl_exchange_check"]["status"] == "timeout"
    assert "not reached" not in r.stdout
    # a check that returns in time passes its value through and leaves the process running
    b = _bench()
    assert b.run_with_watchdog(lambda: 7, 30, None, 0) == 7
