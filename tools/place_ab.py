"""Placement A/B in one process: kg_place over the same workload under several (kernel forms, chunk) settings,
interleaved `--rounds` times, placements checked identical across settings.

  python tools/place_ab.py c2|c3|c5 [--pods N] [--settings 0:16,1:16,1:32] [--rounds 2]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=("c2", "c3", "c5"))
    ap.add_argument("--pods", type=int, default=0)
    ap.add_argument("--settings", default="0:16,1:16")
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    P = a.pods or {"c2": 10_000, "c3": 1_000, "c5": 20_000}[a.which]
    if a.which == "c3":
        cl = synth.make_numa_cluster(100_000, P, seed=3)
    elif a.which == "c5":
        cl = synth.make_rsv_cluster(100_000, P, seed=5)
    else:
        cl = synth.make_cluster(100_000, P, seed=2)
    settings = [tuple(int(x, 0) for x in s.split(":")) for s in a.settings.split(",")]
    ref = None
    res = {s: [] for s in settings}
    for _ in range(a.rounds):
        for forms, chunk in settings:
            cfg = shipped_profile(place_chunk=chunk,
                                  plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota")) \
                if a.which == "c5" else shipped_profile(place_chunk=chunk)
            if a.which == "c3":
                cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
            rows = engine.build_node_rows(cfg, cl)
            pods = engine.build_pod_rows(cfg, cl, np.arange(P))
            with engine.Engine(cfg) as eng:
                eng.set_forms(forms)
                eng.load_snapshot(rows)
                if a.which == "c5":
                    eng.set_reservations(cl.rsv_arr)
                    eng.set_quotas(cl.quota_arr)
                eng.set_pods(pods)
                eng.sync()
                t0 = time.perf_counter()
                nodes, scores = eng.place(cl.now_ns)
                dt = time.perf_counter() - t0
            if ref is None:
                ref = nodes
            assert np.array_equal(nodes, ref), (forms, chunk)
            res[(forms, chunk)].append(P / dt)
    for (forms, chunk), v in res.items():
        print(f"{a.which} forms=0x{forms:x} chunk={chunk}: " + " ".join(f"{x:.0f}" for x in v) + " pods/s", flush=True)


if __name__ == "__main__":
    main()
