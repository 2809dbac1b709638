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
