"""Sharded placement over RCCL at world size 1 (GPU box): the native kg_place_sharded (the chunk loop and the
partial-key ncclAllReduce in C++, dist.native_engine) and dist.place_sharded with the partial-key all_reduce
running through the nccl backend (collective=True), pipelined and not, beside kg_place on the same config-2
batch (a second kg_place run first, for the run-to-run spread).  The merge is a real RCCL launch on the eval stream, so the pipelined rate shows what the per-chunk
collective costs the sequential cycle when it overlaps the resolve.

    python tools/rccl_place_rate.py [pods]
"""
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, ".")
from koordinator_amd import dist as kdist  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", rank=0, world_size=1, device_id=dev)
cl = synth.make_cluster(100_000, P, seed=2)
cfg = shipped_profile()
rows = engine.build_node_rows(cfg, cl)
pods = engine.build_pod_rows(cfg, cl, np.arange(P))
chunk = kdist.place_chunk_of(cfg)

with engine.Engine(cfg) as eng:
    eng.load_snapshot(rows)
    eng.set_pods(pods)
    eng.sync()
    t0 = time.perf_counter()
    ref_nodes, _ = eng.place(cl.now_ns)
    t_one = time.perf_counter() - t0

out = {"kg_place": P / t_one}
with engine.Engine(cfg) as eng:
    eng.load_snapshot(rows)
    eng.set_pods(pods)
    eng.sync()
    t0 = time.perf_counter()
    eng.place(cl.now_ns)
    out["kg_place (again)"] = P / (time.perf_counter() - t0)
for rep in range(2):
    neng = kdist.native_engine(cfg, rows, pods, dev)
    neng.sync()
    t0 = time.perf_counter()
    nodes, _ = neng.place_sharded(cl.now_ns)
    dt = time.perf_counter() - t0
    neng.close()
    assert np.array_equal(nodes, ref_nodes), "native sharded placements differ from kg_place"
    out[f"kg_place_sharded (native RCCL, run {rep})"] = P / dt
for pipeline in (True, False):
    deng = kdist.sharded_engine(cfg, rows, pods, dev)
    kdist.place_sharded(deng, cl.now_ns, dev, chunk=chunk, pipeline=pipeline, collective=True)   # warm-up
    deng.close()
    deng = kdist.sharded_engine(cfg, rows, pods, dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    nodes, _ = kdist.place_sharded(deng, cl.now_ns, dev, chunk=chunk, pipeline=pipeline, collective=True)
    dt = time.perf_counter() - t0
    deng.close()
    assert np.array_equal(nodes, ref_nodes), "sharded placements differ from kg_place"
    out[f"place_sharded(nccl, pipeline={pipeline})"] = P / dt
for k, v in out.items():
    print(f"{k}: {v:.0f} pods/s ({v / out['kg_place']:.2f}x of kg_place)", flush=True)
dist.destroy_process_group()
