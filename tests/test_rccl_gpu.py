"""The RCCL (`nccl` backend) path of the multi-GPU engine, executed on one GPU at world size 1.

The driver's scaling bench runs these collectives over 2–8 MI355X; here they run for real (RCCL, not gloo)
on a one-rank communicator, on the engine's streams, with their results checked against the oracle:
* the bench step's `nccl` branch (bench.py: `all_gather_into_tensor` of the per-pod top-1 keys and a max over
  ranks) and `dist.merge_top1_` (`all_reduce(MAX)` with the sign flip);
* `dist.place_sharded` with the partial-key merge forced through RCCL (`collective=True`), pipelined (chunk
  i + 1 evaluated and merged on the eval stream while chunk i is resolved: kg_place_chunk_resolve_prev) and not.
"""
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

from koordinator_amd import dist as kdist
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def nccl_world1():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        yield dev
    finally:
        dist.destroy_process_group()


def test_rccl_bench_step_and_sharded_placement(nccl_world1):
    dev = nccl_world1
    P = 200
    cl = synth.make_cluster(3_000, P, seed=81)
    cfg = shipped_profile()
    idx = np.arange(P)
    rows = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    m, f, l = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
    t_ref = np.where(m, f.astype(np.int64) + l, -1)
    want = np.where(t_ref.max(axis=1) >= 0, t_ref.argmax(axis=1), -1)
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    for pipeline in (True, False):
        eng = kdist.sharded_engine(cfg, rows, pods, dev)
        try:
            with torch.cuda.stream(eng.torch_stream):
                top1 = torch.zeros(P, dtype=torch.int64, device=dev)
                gathered = torch.zeros((1, P), dtype=torch.int64, device=dev)
                eng.eval_device(cl.now_ns, 0, 0, top1.data_ptr())
                dist.all_gather_into_tensor(gathered.view(-1), top1)   # bench.py's nccl branch
                merged = gathered.max(dim=0).values
                reduced = top1.clone()
                kdist.merge_top1_(reduced)                             # all_reduce(MAX), sign-flipped
                torch.cuda.synchronize(dev)
            for keys in (merged, reduced):
                node, tot = engine.decode_top1(keys.cpu().numpy().view(np.uint64))
                np.testing.assert_array_equal(node, want)
                np.testing.assert_array_equal(tot, t_ref.max(axis=1))
            nodes, scores = kdist.place_sharded(eng, cl.now_ns, dev, chunk=16, pipeline=pipeline, collective=True)
            np.testing.assert_array_equal(nodes, ref_n)
            np.testing.assert_array_equal(scores, ref_s)
        finally:
            eng.close()
