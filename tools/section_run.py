"""One bench section's matrix pass, repeated, for rocprofv3 (kernel trace / PMC passes of a single workload):

  c2_distinct  config-2 nodes, 10k pairwise-distinct pods (k_eval3 plain part)
  c3_eq        config-3, 1k pods of 70 distinct rows (k_eval_numa2 over the distinct rows + k_eq_rows)
  c3_distinct  config-3, 1k pairwise-distinct pods (k_eval_numa2)
  c5_matrix    config-5, 1k batch pods with Reservation + ElasticQuota (plain nodes + k_rsv_eval / k_rsv_reduce)

  python tools/section_run.py <section> [--reps 5] [--nodes 100000]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("section", choices=("c2_distinct", "c3_eq", "c3_distinct", "c5_matrix"))
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--nodes", type=int, default=100_000)
    ap.add_argument("--pods", type=int, default=0)
    a = ap.parse_args()
    import torch

    from koordinator_amd import _native as nat
    from koordinator_amd import engine, synth
    from koordinator_amd.config import shipped_profile

    dev = torch.device("cuda", 0)
    N = a.nodes
    cfg = shipped_profile()
    rsv = quota = None
    if a.section == "c2_distinct":
        P = a.pods or 10_000
        cl = synth.make_cluster(N, 1, seed=2)
        pods_cl = synth.make_cluster(1, P, seed=2, distinct_pods=True)
        rows, prow = engine.build_node_rows(cfg, cl), engine.build_pod_rows(cfg, pods_cl, np.arange(P))
    elif a.section in ("c3_eq", "c3_distinct"):
        P = a.pods or 1_000
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
        cl = synth.make_numa_cluster(N, P, seed=3, distinct_pods=a.section == "c3_distinct")
        rows, prow = engine.build_node_rows(cfg, cl), engine.build_pod_rows(cfg, cl, np.arange(P))
    else:
        P = a.pods or 1_000
        cl = synth.make_rsv_cluster(N, P, seed=5)
        cfg["enabled_plugins"] |= nat.PLUGIN_RESERVATION | nat.PLUGIN_ELASTICQUOTA
        rows, prow = engine.build_node_rows(cfg, cl), engine.build_pod_rows(cfg, cl, np.arange(P))
        rsv, quota = cl.rsv_arr, cl.quota_arr
    eng = engine.Engine(cfg)
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)
    eng.load_snapshot(rows)
    if rsv is not None:
        eng.set_reservations(rsv)
        eng.set_quotas(quota)
    eng.set_pods(prow)
    W = eng.mask_words
    mask = torch.empty((P, W), dtype=torch.int64, device=dev)
    scores = torch.empty((P, W * 64, 2), dtype=torch.uint8, device=dev)
    numa = torch.empty((P, W * 64), dtype=torch.uint8, device=dev) if a.section.startswith("c3") else None
    top1 = torch.zeros(P, dtype=torch.int64, device=dev)
    step = lambda: eng.eval_device(cl.now_ns, mask.data_ptr(), scores.data_ptr(), top1.data_ptr(),
                                   numa.data_ptr() if numa is not None else 0)
    step()
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    t0 = time.perf_counter()
    ev[0].record(stream)
    for _ in range(a.reps):
        step()
    ev[1].record(stream)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / a.reps
    print(f"{a.section}: {P} pods x {N} nodes, {dt * 1e3:.3f} ms per pass (device {ev[0].elapsed_time(ev[1]) / a.reps:.3f} ms), "
          f"distinct rows {len({r.tobytes() for r in prow})}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
