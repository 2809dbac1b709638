"""Source hash of libknn_amd.so: sha256 over the sources it is built from (their paths
relative to this directory and their bytes, in sorted order), first 16 hex digits.

The Makefile bakes it into the library (knn_build_id(), build/knn_build_id.c), and the
tests / smoke() recompute it from the tree they run in: a library that does not match
the sources beside it was not built from them.

usage: python build_id.py   -> prints the id
"""
import glob
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PATTERNS = ("Makefile", "csrc/*.hip", "csrc/*.cpp", "csrc/*.h", "../include/*.h", "../include/*.hpp")


def sources():
    files = set()
    for pat in PATTERNS:
        files.update(os.path.relpath(p, _HERE) for p in glob.glob(os.path.join(_HERE, pat)))
    return sorted(files)


def compute():
    h = hashlib.sha256()
    for rel in sources():
        with open(os.path.join(_HERE, rel), "rb") as f:
            data = f.read()
        h.update(rel.encode() + b"\0" + str(len(data)).encode() + b"\0" + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(compute())
