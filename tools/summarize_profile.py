"""Condense one tools/profile.sh run (rocprofv3 kernel trace + PMC passes) into profiles/<tag>/.

    python tools/summarize_profile.py gpurun_out/prof_<tag> profiles/<tag>

Writes kernel_stats.csv (the rocprofv3 --stats summary, verbatim), pmc_<pass>.csv (the per-dispatch
counter rows of the hot kernel only) and summary.json:
  * per-kernel average duration (ns) from the --kernel-trace --stats pass;
  * per-dispatch averages of every PMC counter of the hot kernel (k_eval*);
  * HBM traffic per launch, corrected as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE and
    WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide streaming read,
    so it is doubled; WRITE_SIZE is taken as is.
bench.py reads summary.json (when its kernel matches) for roofline.traffic.
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict

HOT = "k_eval3"


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main(src: str, dst: str) -> None:
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    kernels = []
    for r in _rows(stats):
        kernels.append({"name": r["Name"][:160], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                        "percent": float(r["Percentage"])})
    # matrix mode launches one k_eval3 per class kind present in the batch: a "launch" of the hot path
    # is one pass = one dispatch of every kind, so its duration and counters are the sums over kinds
    parts = [k for k in kernels if HOT in k["name"]]
    hot = None
    if parts:
        calls = min(k["calls"] for k in parts)
        hot = {"name": " + ".join(k["name"].split("(")[0] for k in parts), "calls": calls,
               "avg_ns": sum(k["avg_ns"] for k in parts), "percent": sum(k["percent"] for k in parts),
               "parts": parts}
    # the forms / kinds run on two streams: their durations overlap, so the pass time is the
    # wall span from the first kind's start to the last kind's end, taken per pass from the kernel trace
    trace = os.path.join(src, "trace", "trace_kernel_trace.csv")
    if hot and os.path.exists(trace):
        disp = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in _rows(trace) if HOT in r["Kernel_Name"])
        k = len(parts)
        spans = [max(e for _, e in disp[i:i + k]) - disp[i][0] for i in range(0, len(disp) - k + 1, k)]
        if spans:
            hot["sum_of_kinds_ns"] = hot["avg_ns"]
            hot["pass_spans_ns"] = spans
            hot["avg_ns"] = sum(spans) / len(spans)
            hot["avg_ns_source"] = "mean wall span per pass (first kind start → last kind end) from the kernel trace"
    pmc = {}
    for name in sorted(os.listdir(src)):
        d = os.path.join(src, name)
        if not (name.startswith("pmc_") and os.path.isdir(d)):
            continue
        f = os.path.join(d, f"{name}_counter_collection.csv")
        if not os.path.exists(f):
            continue
        rows = [r for r in _rows(f) if HOT in r["Kernel_Name"]]
        with open(os.path.join(dst, f"{name}.csv"), "w", newline="") as out:
            if rows:
                w = csv.DictWriter(out, fieldnames=list(rows[0].keys()))
                w.writeheader()
                w.writerows(rows)
        acc = defaultdict(lambda: defaultdict(list))   # counter -> kernel -> per-dispatch values
        for r in rows:
            acc[r["Counter_Name"]][r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, per_kernel in acc.items():   # per pass: Σ over kinds of the per-dispatch average
            pmc[k] = sum(sum(v) / len(v) for v in per_kernel.values())
    traffic = None
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        traffic = {"fetch_bytes": 2 * pmc["FETCH_SIZE"] * 1024, "write_bytes": pmc["WRITE_SIZE"] * 1024}
        traffic["total_bytes"] = traffic["fetch_bytes"] + traffic["write_bytes"]
    summary = {"hot_kernel": hot, "kernels": kernels, "pmc_per_dispatch": pmc, "hbm_traffic_per_launch": traffic}
    if hot and "GRBM_GUI_ACTIVE" in pmc and len(hot["parts"]) == 1:
        # GRBM_GUI_ACTIVE counts GPU-busy cycles of each of the 8 XCDs over the dispatch; with more than one
        # concurrent launch per pass (two streams) the per-dispatch counts overlap in time and no clock follows
        summary["effective_clock_ghz"] = pmc["GRBM_GUI_ACTIVE"] / 8 / hot["avg_ns"]
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({"hot": hot, "traffic": traffic}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
