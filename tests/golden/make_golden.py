"""Capture golden fixtures from the REFERENCE (run in the build container only).

Runs oracle/_ref/ref_capture -- the reference's own main.cpp KNN(),
computeConfusionMatrix() and computeAccuracy() (main.cpp:25,87,102), compiled
from /root/reference by oracle/Makefile -- on every dataset x k and writes:

  pred_<ds>_k<k>.txt   one "%d\\n" prediction per query (SURVEY.md 8c sha256 contract)
  cm_<ds>_k<k>.txt     accuracy line + confusion-matrix rows as printed by the harness
  topk_<ds>_k<k>.bin   int32 {nq, k} then nq*k records {uint32 dist_bits, int32 train_idx}
  manifest.json        sha256 of every prediction file, accuracy, shapes

Usage:  python tests/golden/make_golden.py   (after `make -C oracle`)
"""
import concurrent.futures as cf
import hashlib
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
DATA = os.path.join(REPO, "tests", "data")
CAPTURE = os.path.join(REPO, "oracle", "_ref", "ref_capture")
DATASETS = ["small", "medium", "large"]
KS = [1, 3, 5, 10, 32, 100]


def run(ds, k):
    pred = os.path.join(HERE, f"pred_{ds}_k{k}.txt")
    topk = os.path.join(HERE, f"topk_{ds}_k{k}.bin")
    out = subprocess.run(
        [CAPTURE, os.path.join(DATA, f"{ds}-train.arff"), os.path.join(DATA, f"{ds}-test.arff"),
         str(k), pred, topk],
        check=True, capture_output=True, text=True).stdout
    with open(os.path.join(HERE, f"cm_{ds}_k{k}.txt"), "w") as f:
        f.write(out)
    with open(pred, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    acc = float(out.split()[1])
    return ds, k, sha, acc


def main():
    if not os.path.exists(CAPTURE):
        sys.exit("build oracle/_ref/ref_capture first: make -C oracle")
    manifest = {}
    with cf.ThreadPoolExecutor(max_workers=6) as ex:
        for ds, k, sha, acc in ex.map(lambda a: run(*a), [(d, k) for d in DATASETS for k in KS]):
            manifest[f"{ds}_k{k}"] = {"dataset": ds, "k": k, "sha256": sha, "accuracy": acc}
            print(ds, k, sha, acc)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
