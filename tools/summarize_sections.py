"""Condense a tools/profile_sections.sh run into one JSON: per section, the rocprofv3 --stats rows of its kernels and
the per-dispatch averages of every PMC counter of the kernels that take ≥ 5 % of the section's time
(WRITE_SIZE / FETCH_SIZE in KiB as rocprofv3 reports them; FETCH_SIZE doubled for gfx950 as in summarize_profile.py).

    python tools/summarize_sections.py gpurun_out/sec_<tag> profiles/<tag>/sections.json
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main(src, dst):
    out = {}
    for sec in sorted(os.listdir(src)):
        d = os.path.join(src, sec)
        stats = os.path.join(d, "trace", "trace_kernel_stats.csv")
        if not os.path.exists(stats):
            continue
        kernels = [{"name": r["Name"][:120], "calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                    "percent": float(r["Percentage"])} for r in csv.DictReader(open(stats))]
        hot = [k["name"][:40] for k in kernels if k["percent"] >= 5.0]
        pmc = defaultdict(lambda: defaultdict(list))
        for p in ("pmc_sq", "pmc_fetch", "pmc_write"):
            f = os.path.join(d, p, p + "_counter_collection.csv")
            if not os.path.exists(f):
                continue
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"][:40]
                if name in hot:
                    pmc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        counters = {}
        for name, cs in pmc.items():
            counters[name] = {}
            for c, v in cs.items():
                avg = sum(v) / len(v)
                if c == "FETCH_SIZE":
                    counters[name]["fetch_bytes"] = avg * 1024 * 2
                elif c == "WRITE_SIZE":
                    counters[name]["write_bytes"] = avg * 1024
                else:
                    counters[name][c] = avg
        out[sec] = {"kernels": kernels, "pmc_per_dispatch": counters}
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
