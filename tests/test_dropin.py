"""The drop-in boundary, proven on the reference's OWN drivers: main.cpp, multi-thread.cpp
and mpi.cpp, patched by oracle/dropin.py (libarff includes -> include/knn_arff.hpp or
knn_compat_threads.hpp; their distance / KNN / computeConfusionMatrix / computeAccuracy
definitions deleted, nothing else touched) and linked against libknn_amd.so by
oracle/Makefile (_ref/dropin_*).  Their argv handling, timed region, pthreads / MPI
calls and printed line are the reference's; the KNN they call is this library's.  The
GPU tests run them on the reference's datasets and check the printed line and the
predictions (tapped at computeConfusionMatrix by oracle/dropin_tap.cpp) against the
golden sha256 captured from the unmodified reference (anchors: main.cpp:114-147,
multi-thread.cpp:133-208, mpi.cpp:119-206)."""
import hashlib
import os
import re
import subprocess
import sys

import pytest

from conftest import DATA, ORACLE_DIR, REPO, golden_manifest

REF = "/root/reference"
REF_DIR = os.path.join(ORACLE_DIR, "_ref")
MPIEXEC = "/opt/conda/bin/mpiexec"
LINE = re.compile(r"^The (-?\d+)-NN classifier for (\d+) test instances on (\d+) train instances "
                  r"required (\d+) ms CPU time\. Accuracy was (\d\.\d{4})$")
# the definitions the patch deletes (1-based inclusive line ranges of the reference files)
EXPECTED_CUTS = {
    "main.cpp": [(14, 23), (25, 85), (87, 100), (102, 112)],
    "multi-thread.cpp": [(18, 24), (26, 35), (37, 104), (106, 119), (121, 131)],
    "mpi.cpp": [(15, 24), (26, 90), (92, 105), (107, 117)],
}


def _exe(name):
    p = os.path.join(REF_DIR, name)
    if not os.path.exists(p):
        pytest.skip(f"{p} not built (oracle/Makefile needs the reference sources)")
    return p


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference sources absent (GPU box)")
def test_dropin_patch_touches_only_the_definitions(tmp_path):
    sys.path.insert(0, ORACLE_DIR)
    try:
        import dropin
    finally:
        sys.path.pop(0)
    for name, cuts in EXPECTED_CUTS.items():
        with open(os.path.join(REF, name)) as f:
            text = f.read()
        inc, names = dropin.DRIVERS[name]
        out, deleted = dropin.patch(text, inc, names)
        assert deleted == cuts, name
        # every line outside the cuts and the two libarff includes survives, in order
        keep = [ln for i, ln in enumerate(text.splitlines(), 1)
                if not any(a <= i <= b for a, b in cuts) and not dropin.LIBARFF_INCLUDE.match(ln)]
        got = [ln for ln in out.splitlines() if not ln.startswith("// drop-in:") and not ln.startswith("#include \"knn_")]
        assert got == keep, name
        assert f'#include "{inc}"' in out


@pytest.mark.parametrize("exe,usage", [
    ("dropin_main", "Usage: ./main datasets/train.arff datasets/test.arff k"),
    ("dropin_multi-thread", "Usage: ./multi-thread datasets/train.arff datasets/test.arff k numThreads"),
])
def test_dropin_binaries_load_the_library(exe, usage):
    """The patched drivers link libknn_amd.so and run their own argv check (no GPU needed)."""
    r = subprocess.run([_exe(exe)], capture_output=True, text=True, timeout=60)
    assert r.stdout.strip().splitlines()[0] == usage, r.stdout


def _check(r, pred_file, ds, k):
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("The ")]
    assert len(lines) == 1, r.stdout
    m = LINE.match(lines[0])
    g = golden_manifest()[f"{ds}_k{k}"]
    assert m and int(m.group(1)) == k and m.group(5) == f"{g['accuracy']:.4f}", lines[0]
    with open(pred_file, "rb") as f:
        assert hashlib.sha256(f.read()).hexdigest() == g["sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("ds,k", [("large", 5), ("medium", 3), ("small", 1)])
def test_dropin_main_golden(tmp_path, ds, k):
    out = tmp_path / "pred.txt"
    r = subprocess.run([_exe("dropin_main"), f"{DATA}/{ds}-train.arff", f"{DATA}/{ds}-test.arff", str(k)],
                       capture_output=True, text=True, timeout=120, env=dict(os.environ, KNN_DROPIN_PRED_OUT=str(out)))
    _check(r, out, ds, k)


@pytest.mark.gpu
@pytest.mark.parametrize("ds,k,threads", [("large", 5, 4), ("medium", 10, 3)])
def test_dropin_multi_thread_golden(tmp_path, ds, k, threads):
    out = tmp_path / "pred.txt"
    r = subprocess.run([_exe("dropin_multi-thread"), f"{DATA}/{ds}-train.arff", f"{DATA}/{ds}-test.arff", str(k),
                        str(threads)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, KNN_DROPIN_PRED_OUT=str(out)))
    _check(r, out, ds, k)


@pytest.mark.gpu
def test_dropin_mpi_golden(tmp_path):
    if not os.path.exists(MPIEXEC):
        pytest.skip("MPICH absent")
    out = tmp_path / "pred.txt"
    r = subprocess.run([MPIEXEC, "-n", "2", _exe("dropin_mpi"), f"{DATA}/large-train.arff",
                        f"{DATA}/large-test.arff", "5"], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, KNN_DROPIN_PRED_OUT=str(out)))
    _check(r, out, "large", 5)
