"""Placement throughput vs kg_place chunk size on the config-2 cluster, or config 3 (NodeNUMAResource)
with a second argument "c3" (one GPU)."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
C3 = len(sys.argv) > 2 and sys.argv[2] == "c3"
cl = synth.make_numa_cluster(100_000, P, seed=3) if C3 else synth.make_cluster(100_000, P, seed=2)
rows = None
ref = None
for chunk in ((2, 4, 8, 16) if C3 else (4, 8, 12, 16, 24, 32)):
    cfg = shipped_profile(place_chunk=chunk)
    if C3:
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    if rows is None:
        rows = engine.build_node_rows(cfg, cl)
        pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(rows)
        eng.set_pods(pods)
        eng.sync()
        t0 = time.perf_counter()
        nodes, scores = eng.place(cl.now_ns)
        dt = time.perf_counter() - t0
    if ref is None:
        ref = nodes
    print(f"chunk {chunk}: {dt:.3f} s, {P / dt:.0f} pods/s, same placements: {bool((nodes == ref).all())}", flush=True)
