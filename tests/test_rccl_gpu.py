"""The RCCL (`nccl` backend) path of the multi-GPU engine, executed on one GPU at world size 1.

The driver's scaling bench runs these collectives over 2–8 MI355X; here they run for real (RCCL, not gloo)
on a one-rank communicator, on the engine's streams, with their results checked against the oracle:
* the bench step's `nccl` branch (bench.py: `all_gather_into_tensor` of the per-pod top-1 keys and a max over
  ranks) and `dist.merge_top1_` (`all_reduce(MAX)` with the sign flip);
* `dist.place_sharded` with the partial-key merge forced through RCCL (`collective=True`), pipelined (chunk
  i + 1 evaluated and merged on the eval stream while chunk i is resolved: kg_place_chunk_resolve_prev) and not;
* the native sharded placement (`kg_place_sharded` on the engine's own RCCL communicator, `dist.native_engine`),
  sequential and pipelined, with Reservation + ElasticQuota, and with cpuset pods (the host Reserve replicated).
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


def _native_place(cfg, rows, pods, dev, cl, **kw):
    eng = kdist.native_engine(cfg, rows, pods, dev, **kw)
    try:
        return eng.place_sharded(cl.now_ns)
    finally:
        eng.close()


@pytest.mark.parametrize("kind", ["fit_la", "numa", "rsv_quota"])
def test_native_sharded_placement_world1(nccl_world1, kind):
    """kg_place_sharded (the chunk loop, the partial-key ncclAllReduce and the replicated resolve in C++) on a
    one-rank RCCL communicator of its own: placements and scores equal the oracle's sequential cycle, for the
    sequential form (Fit + LoadAware, Reservation + ElasticQuota) and the pipelined one (NodeNUMAResource: the
    merge on the eval stream beside the resolve)."""
    from koordinator_amd import _native as nat
    from rsv_cases import rsv_cluster
    dev = nccl_world1
    P = 240
    kw = {}
    if kind == "fit_la":
        cl = synth.make_cluster(3_000, P, seed=83)
        cfg = shipped_profile()
    elif kind == "numa":
        cl = synth.make_numa_cluster(2_000, P, seed=84)
        cfg = shipped_profile()
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    else:
        cl = rsv_cluster(2_500, P, seed=85, n_quotas=8, quota_ratio=0.6)
        cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"))
        kw = dict(reservations=cl.rsv_arr, quotas=cl.quota_arr)
    idx = np.arange(P)
    rows = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    nodes, scores = _native_place(cfg, rows, pods, dev, cl, **kw)
    if kind == "rsv_quota":
        ref_n, ref_s, _, _ = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    else:
        ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)


def test_native_sharded_placement_binds_cpusets(nccl_world1):
    """Cpuset pods on the native sharded path: the host Reserve (the CPU accumulator on the node's CPU table) runs
    after the replicated resolve, identically on every rank; placements, scores and CPUs equal the oracle's."""
    from bind_cases import make_bind_cluster
    from koordinator_amd import _native as nat
    from reserve_cycle import cpu_tables
    dev = nccl_world1
    cl, view, idx = make_bind_cluster(300, 200, 21, numa_frac=0.35)
    cfg = shipped_profile(place_chunk=16)
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    rows = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, idx)
    eng = kdist.native_engine(cfg, rows, pods, dev)
    try:
        eng.set_cpus(view)
        nodes, scores = eng.place_sharded(cl.now_ns)
        tabs = cpu_tables(view)
        got = view.cpu_arr.copy()
        for j, (first, n, _, _) in tabs.items():
            got[first:first + n] = eng.download_cpus(j, n)
    finally:
        eng.close()
    ref_nodes, ref_scores, ref_cpus = oracle.schedule_cpus(cfg, view, np.asarray(idx), cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(got, ref_cpus)
