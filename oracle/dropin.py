"""dropin.py -- the drop-in patch of the reference's own drivers, as a recipe.

TEST INFRASTRUCTURE ONLY.  Reads main.cpp / multi-thread.cpp / mpi.cpp where they lie
under the reference checkout and writes patched copies into oracle/_ref/dropin/ (git-
ignored: no reference text enters the repository).  The patch is what INTEGRATION.md
describes, applied mechanically:

  * the two libarff includes (main.cpp:8-9, multi-thread.cpp:8-9, mpi.cpp:8-9) become
    `#include "knn_arff.hpp"` (main, mpi) or `#include "knn_compat_threads.hpp"`
    (multi-thread);
  * the driver's own definitions of distance / KNN / computeConfusionMatrix /
    computeAccuracy (main.cpp:14-112, multi-thread.cpp:26-131, mpi.cpp:15-117) and
    multi-thread.cpp's `struct arguments` (:18-24, declared by the compat header) are
    deleted -- each definition from its signature line through its matching brace;
  * everything else (argv parsing, the timed region, threads / MPI calls, the printed
    line) is the reference's, byte for byte.

The result is linked against libknn_amd.so (oracle/Makefile, targets dropin_*) and run by
tests/test_dropin.py against the golden predictions.

usage: python dropin.py REF_DIR OUT_DIR
"""
import os
import re
import sys

DRIVERS = {
    # driver: (replacement include, definitions to delete)
    "main.cpp": ("knn_arff.hpp", ("distance", "KNN", "computeConfusionMatrix", "computeAccuracy")),
    "multi-thread.cpp": ("knn_compat_threads.hpp",
                         ("distance", "KNN", "computeConfusionMatrix", "computeAccuracy", "struct arguments")),
    "mpi.cpp": ("knn_arff.hpp", ("distance", "KNN", "computeConfusionMatrix", "computeAccuracy")),
}
LIBARFF_INCLUDE = re.compile(r'^\s*#include\s+"libarff/arff_(parser|data)\.h"\s*$')


def _starts_definition(line, names):
    for n in names:
        if n.startswith("struct "):
            if re.match(r"^\s*" + re.escape(n) + r"\s*\{?\s*$", line):
                return True
        elif re.match(r"^[A-Za-z_][\w\s\*]*?[\s\*]" + re.escape(n) + r"\s*\(", line):
            return True
    return False


def patch(text, include, names):
    lines = text.splitlines(keepends=True)
    out, i, replaced, deleted = [], 0, False, []
    while i < len(lines):
        ln = lines[i]
        if LIBARFF_INCLUDE.match(ln):
            if not replaced:
                out.append(f'#include "{include}"  // drop-in: was the libarff includes\n')
                replaced = True
            i += 1
            continue
        if _starts_definition(ln, names):
            depth, seen, j = 0, False, i
            while j < len(lines):
                for ch in lines[j]:
                    if ch == "{":
                        depth, seen = depth + 1, True
                    elif ch == "}":
                        depth -= 1
                j += 1
                if seen and depth == 0:
                    break
            deleted.append((i + 1, j))
            out.append(f"// drop-in: lines {i + 1}-{j} (the driver's own definition) removed\n")
            i = j
            continue
        out.append(ln)
        i += 1
    if not replaced:
        raise SystemExit("libarff includes not found")
    return "".join(out), deleted


def main(argv):
    ref, dst = argv[1], argv[2]
    os.makedirs(dst, exist_ok=True)
    for name, (include, names) in DRIVERS.items():
        src = os.path.join(ref, name)
        if not os.path.exists(src):
            continue
        with open(src) as f:
            text, deleted = patch(f.read(), include, names)
        if len(deleted) < len(names):
            raise SystemExit(f"{name}: expected {len(names)} definitions, found {deleted}")
        with open(os.path.join(dst, name), "w") as f:
            f.write(text)
        print(f"{name}: removed lines {deleted}")


if __name__ == "__main__":
    main(sys.argv)
