"""Generates tests/golden/fullsize_placements.npz: the oracle's sequential cycle over the whole bench bursts
that are too long to re-run inside the GPU suite.

* config 3: all 1,000 pods of the bench's NodeNUMAResource placement (seed 3, 100k nodes), kgo_schedule_parallel;
* config 5: all 100,000 pods of the bench's Reservation + ElasticQuota burst (seed 5, 100k nodes),
  kgo_schedule2_parallel, with the reservation and quota states after the last Reserve.

Each case stores a SHA-256 digest of the engine inputs it was computed from (node, pod, reservation and quota
rows), so tests/test_fullsize_place_gpu.py refuses a stale fixture instead of comparing against it.  The
oracle's per-node loop runs on threads; the cycle (Reserve order, reductions) is the sequential one.

    python tests/golden/make_fullsize_placements.py [--workers N] [--only c3|c5]

Takes ≈ 35 min on 8 host threads (config 5 dominates: ≈ 19 ms of node loop per pod).
"""
import argparse
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402
from oracle import oracle  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize_placements.npz")
RSV_EQ = ("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota")


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8).tobytes())
    return h.hexdigest()


def c3_case():
    """(cfg, cluster, node rows, pod rows) of the config-3 placement burst."""
    N, P = 100_000, 1_000
    cl = synth.make_numa_cluster(N, P, seed=3)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    return cfg, cl, engine.build_node_rows(cfg, cl), engine.build_pod_rows(cfg, cl, np.arange(P))


def c5_case():
    """(cfg, cluster, node rows, pod rows) of the config-5 burst."""
    N, P = 100_000, 100_000
    cl = synth.make_rsv_cluster(N, P, seed=5)
    cfg = shipped_profile(plugins=RSV_EQ)
    return cfg, cl, engine.build_node_rows(cfg, cl), engine.build_pod_rows(cfg, cl, np.arange(P))


def c3_digest(nrows, prows) -> str:
    return digest(nrows, prows)


def c5_digest(cl, nrows, prows) -> str:
    return digest(nrows, prows, cl.rsv_arr, cl.quota_arr)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--only", choices=("c3", "c5"))
    a = ap.parse_args()
    out = dict(np.load(OUT)) if os.path.exists(OUT) else {}
    if a.only in (None, "c3"):
        cfg, cl, nrows, prows = c3_case()
        t = time.time()
        nodes, scores = oracle.schedule_parallel(cfg, cl, np.arange(len(prows)), cl.now_ns, a.workers)
        print(f"config 3: {len(nodes)} pods in {time.time() - t:.0f} s, {(nodes >= 0).sum()} placed", flush=True)
        out.update(c3_digest=np.array(c3_digest(nrows, prows)), c3_nodes=nodes, c3_scores=scores)
    if a.only in (None, "c5"):
        cfg, cl, nrows, prows = c5_case()
        t = time.time()
        nodes, scores, rsv, q = oracle.schedule2(cfg, cl, np.arange(len(prows)), cl.now_ns, workers=a.workers)
        print(f"config 5: {len(nodes)} pods in {time.time() - t:.0f} s, {(nodes >= 0).sum()} placed", flush=True)
        out.update(c5_digest=np.array(c5_digest(cl, nrows, prows)), c5_nodes=nodes, c5_scores=scores,
                   c5_rsv_n_assigned=rsv["n_assigned"], c5_rsv_allocated=rsv["allocated"]["v"],
                   c5_quota_used=q["used"]["v"], c5_quota_np_used=q["non_preemptible_used"]["v"])
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
