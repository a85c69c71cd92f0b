"""Debug helper: 2-rank sharded placement on one GPU vs single-engine kg_place (prints mismatches)."""
import os
import socket
import sys

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from koordinator_amd import dist as kdist  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402


def worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cl = synth.make_cluster(5_000, 300, seed=71)
    cfg = shipped_profile()
    idx = np.arange(300)
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    eng = kdist.sharded_engine(cfg, nodes, pods, dev)
    P, T = eng.n_pods, eng.num_tiles
    part = torch.zeros((64, T), dtype=torch.int32, device=dev)
    eng.chunk_eval(cl.now_ns, 0, 64, part.data_ptr())
    torch.cuda.synchronize()
    local = part.clone()
    kdist.merge_partials_(part)
    torch.cuda.synchronize()
    with engine.Engine(cfg) as e1:
        e1.load_snapshot(nodes)
        e1.set_pods(pods)
        full = torch.zeros((64, T), dtype=torch.int32, device=dev)
        e1.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        e1.chunk_eval(cl.now_ns, 0, 64, full.data_ptr())
        torch.cuda.synchronize()
        ref_n, ref_s = e1.place(cl.now_ns)
    print(rank, "shard", eng.shard, "local nonzero tiles", (local != 0).sum(dim=0).tolist(), flush=True)
    print(rank, "merged==full", bool((part == full).all()), "diff count", int((part != full).sum()), flush=True)
    eng.close()
    got_n, got_s = kdist.place(cfg, nodes, pods, cl.now_ns, device=dev)
    bad = np.nonzero((got_n != ref_n) | (got_s != ref_s))[0]
    print(rank, "placement mismatches", len(bad), bad[:5], got_n[bad[:5]], ref_n[bad[:5]], got_s[bad[:5]],
          ref_s[bad[:5]], flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(worker, args=(2, port), nprocs=2)
