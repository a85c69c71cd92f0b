"""Placement throughput of kg_place vs the chunk size on the config-2 workload (10k pods x 100k nodes,
shipped profile), one GPU.  Placements are the sequential cycle's at every chunk size (asserted equal);
only the number of chunk evaluations / resolves — and in the sharded path the number of collectives —
changes.  Prints one JSON line per chunk size."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from koordinator_amd import engine, synth
    from koordinator_amd.config import shipped_profile

    P, N = int(os.environ.get("SWEEP_PODS", "10000")), int(os.environ.get("SWEEP_NODES", "100000"))
    cl = synth.make_cluster(N, P, seed=2)
    ref = None
    for chunk in (8, 16, 32, 64):
        cfg = shipped_profile(place_chunk=chunk)
        rows = engine.build_node_rows(cfg, cl)
        with engine.Engine(cfg) as eng:
            eng.load_snapshot(rows)
            eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
            eng.place(cl.now_ns)            # warm-up (module load, scratch)
            eng.load_snapshot(rows)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            nodes, _ = eng.place(cl.now_ns)
            dt = time.perf_counter() - t0
        if ref is None:
            ref = nodes
        assert (nodes == ref).all(), f"chunk {chunk} placements differ"
        print(json.dumps({"chunk": chunk, "pods": P, "nodes": N, "seconds": round(dt, 4),
                          "pods_placed_per_s": round(P / dt, 1), "chunks": -(-P // chunk)}), flush=True)


if __name__ == "__main__":
    main()
