"""Summarise the rocprofv3 outputs of scripts/profile_bench.sh into profiles/.

    python scripts/summarize_profile.py TAG [gpurun_out] [CONFIG] [PROF_TAG]

Writes profiles/TAG_kernel_stats.csv (the --stats summary as produced),
profiles/TAG_pmc_traffic.json (per-launch HBM bytes of k_gemm_filter with the gfx950
FETCH_SIZE x2 correction, MFMA busy fraction, effective clock); the per-dispatch counter dump
TAG_pmc_counters.csv stays beside the raw outputs (gpurun_out/, scratch: only the summaries are
evidence).
Rules (MI355X_MICROARCH.md, HBM section): FETCH_SIZE/WRITE_SIZE are in KiB;
FETCH_SIZE reads 1/2 of the bytes of a wide coalesced stream on gfx950 -> double it;
WRITE_SIZE is exact for 16-B streaming stores.  Effective clock = GRBM_GUI_ACTIVE / 8 / wall.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out")
    pt = sys.argv[4] if len(sys.argv) > 4 else "prof"  # profile_bench.sh PROF_TAG
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, pt + "_trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_kernel_stats.csv"))
    # durations per kernel from the trace
    dur = defaultdict(list)
    with open(os.path.join(src, pt + "_trace", "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    counters = defaultdict(lambda: defaultdict(list))
    rows_out = []
    for p in (pt + "_fetch", pt + "_write", pt + "_sq", pt + "_lds"):
        path = os.path.join(src, p, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                v = float(r["Counter_Value"])
                wall = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                counters[k][r["Counter_Name"]].append((v, wall))
                rows_out.append({"pass": p, "kernel": k, "counter": r["Counter_Name"], "value": v,
                                 "wall_s": wall})
    with open(os.path.join(src, f"{tag}_pmc_counters.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["pass", "kernel", "counter", "value", "wall_s"])
        w.writeheader()
        w.writerows(rows_out)

    def mean(xs):
        return sum(xs) / len(xs) if xs else None

    # the bench workload these counters were taken on: bench.py's own key (pmc_key), from the
    # JSON line of the trace pass; argv[3] only when that line is missing
    key = sys.argv[3] if len(sys.argv) > 3 else "A"
    try:
        with open(os.path.join(src, pt + "_trace.log")) as f:
            line = [l for l in f.read().splitlines() if l.startswith("{")][-1]
        key = json.loads(line).get("pmc_key", key)
    except (OSError, IndexError, ValueError):
        pass
    out = {"tag": tag, "config": key}
    # the filter launch that did the work: the matching kernel with the longest trace time
    # (AUTO's gated re-run launches the split filter, which exits at once)
    cands = [k for k in counters if "k_gemm_filter" in k or "k_gemm_fused" in k]
    if not cands:  # the direct-form workloads (config L): the direct kernel
        cands = [k for k in counters if "k_direct" in k]
    cands.sort(key=lambda k: sum(dur.get(k, [0.0])))
    for k in cands[-1:]:
        c = counters[k]
        fetch = mean([v for v, _ in c.get("FETCH_SIZE", [])])
        write = mean([v for v, _ in c.get("WRITE_SIZE", [])])
        gui = c.get("GRBM_GUI_ACTIVE", [])
        busy = mean([v for v, _ in c.get("SQ_VALU_MFMA_BUSY_CYCLES", [])])
        # quad-cycle counters (MI355X_MICROARCH.md): fractions of SQ_WAVE_CYCLES
        wave = mean([v for v, _ in c.get("SQ_WAVE_CYCLES", [])])
        waits = {n: mean([v for v, _ in c.get(n, [])]) for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
        mfma = mean([v for v, _ in c.get("SQ_INSTS_MFMA", [])])
        valu = mean([v for v, _ in c.get("SQ_INSTS_VALU", [])])
        clk = mean([v / 8.0 / w for v, w in gui]) if gui else None
        wall = mean([w for _, w in gui]) if gui else None
        simds = 256 * 4
        out.update({
            "kernel": k,
            "fetch_kib_raw": fetch,
            "write_kib_raw": write,
            "gemm_filter_read_bytes_per_launch": 2.0 * fetch * 1024 if fetch else None,
            "gemm_filter_write_bytes_per_launch": write * 1024 if write else None,
            "gemm_filter_bytes_per_launch": (2.0 * fetch + write) * 1024 if fetch and write else None,
            "effective_clock_ghz": clk / 1e9 if clk else None,
            "mfma_instructions": mfma,
            "valu_instructions": valu,
            "valu_per_mfma": valu / mfma if valu and mfma else None,
            "mfma_busy_frac": busy / (simds * clk * wall) if busy and clk and wall else None,
            "trace_avg_ms": 1e3 * mean(dur.get(k, [])) if dur.get(k) else None,
        })
        for n, v in waits.items():
            if v is not None and wave:
                out[n.lower() + "_frac"] = v / wave
        # every counter of the filter launch, averaged over its launches
        out["counters"] = {n: mean([v for v, _ in vals]) for n, vals in sorted(c.items())}
    with open(os.path.join(prof, f"{tag}_pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    # the index bench.py reads (pmc_traffic): the newest summary per workload key (a study
    # build's profile, KNN_PMC_NO_INDEX=1, stays out of it)
    if os.environ.get("KNN_PMC_NO_INDEX") == "1":
        print(json.dumps(out, indent=1))
        return
    idx_path = os.path.join(prof, "pmc_latest.json")
    try:
        with open(idx_path) as f:
            idx = json.load(f)
    except (OSError, ValueError):
        idx = {}
    idx[key] = {"tag": tag, "file": f"profiles/{tag}_pmc_traffic.json",
                "gemm_filter_bytes_per_launch": out.get("gemm_filter_bytes_per_launch"),
                "trace_avg_ms": out.get("trace_avg_ms"), "kernel": out.get("kernel")}
    with open(idx_path, "w") as f:
        json.dump(idx, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
