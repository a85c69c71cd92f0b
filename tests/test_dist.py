"""Multi-rank (node-sharded) paths, world size 2.

CPU (gloo): the placement protocol of koordinator_amd/dist.py — tile-aligned node shards, the
per-(pod, tile) partial-key merge over the group and the replicated sequential resolve — driven with the
numpy mirror of the engine's chunk API (tests/rows_ref.py), must reproduce the oracle's sequential
cycle; the matrix-mode top-1 merge must equal the single-rank best node.

GPU: two processes share cuda:0 (gloo moves the tensors), each with the HIP engine restricted to its
shard; placements and merged top-1 keys must equal the oracle.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from koordinator_amd import dist as kdist
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def test_shard_ranges_cover_the_snapshot():
    for n in (1, 1023, 1024, 3000, 100_000):
        for world in (1, 2, 3, 8):
            rs = [kdist.shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (b0, e0), (b1, e1) in zip(rs, rs[1:]):
                assert e0 == b1
            assert all((b % 1024 == 0 or b == e) and b <= e for b, e in rs)


def _cpu_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, HERE)
    from oracle import oracle
    from rows_ref import RowsBackend, rows_eval

    _init(rank, world, port)
    try:
        cl = synth.make_cluster(2_600, 90, seed=61, no_metric_frac=0.1)
        cfg = shipped_profile()
        idx = np.arange(90)
        nodes = engine.build_node_rows(cfg, cl)
        pods = engine.build_pod_rows(cfg, cl, idx)
        shard = kdist.shard_range(len(nodes), rank, world)
        # placement: sharded chunk eval + merged partials + replicated resolve
        be = RowsBackend(cfg, nodes, pods, shard)
        got_n, got_s = kdist.place_sharded(be, cl.now_ns, torch.device("cpu"), chunk=16)
        ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
        # matrix mode: local best key of the shard, merged across ranks
        lo, hi = shard
        m, f, l = rows_eval(cfg, nodes[lo:hi], pods, cl.now_ns)
        tot = np.where(m, f + l, -1)
        keys = np.zeros(len(pods), np.uint64)
        if hi > lo:
            j = tot.argmax(axis=1)
            best = tot[np.arange(len(pods)), j]
            keys = np.where(best >= 0, ((best + 1).astype(np.uint64) << np.uint64(32)) |
                            (np.uint64(0xFFFFFFFF) - (lo + j).astype(np.uint64)), np.uint64(0))
        t = torch.from_numpy(keys.view(np.int64).copy())
        kdist.merge_top1_(t)
        merged = t.numpy().view(np.uint64)
        m_all, f_all, l_all = rows_eval(cfg, nodes, pods, cl.now_ns)
        tot_all = np.where(m_all, f_all + l_all, -1)
        want = tot_all.argmax(axis=1)
        got_node = np.where(merged != 0, (0xFFFFFFFF - (merged & np.uint64(0xFFFFFFFF))).astype(np.int64), -1)
        q.put((rank, np.array_equal(got_n, ref_n) and np.array_equal(got_s, ref_s),
               np.array_equal(got_node, np.where(tot_all.max(axis=1) >= 0, want, -1))))
    finally:
        dist.destroy_process_group()


def test_sharded_placement_protocol_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_cpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, placed_ok, top1_ok in res:
        assert placed_ok, f"rank {rank}: sharded placement differs from the sequential oracle"
        assert top1_ok, f"rank {rank}: merged top-1 differs from the single-rank best node"


def _gpu_worker(rank, world, port, q):
    from oracle import oracle

    _init(rank, world, port)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cl = synth.make_cluster(5_000, 300, seed=71)
        cfg = shipped_profile()
        idx = np.arange(300)
        nodes = engine.build_node_rows(cfg, cl)
        pods = engine.build_pod_rows(cfg, cl, idx)
        got_n, got_s = kdist.place(cfg, nodes, pods, cl.now_ns, device=dev)
        ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
        # matrix mode on the shard + top-1 merge
        eng = kdist.sharded_engine(cfg, nodes, pods, dev)
        with torch.cuda.stream(eng.torch_stream):
            top1 = torch.zeros(len(idx), dtype=torch.int64, device=dev)
            eng.eval_device(cl.now_ns, 0, 0, top1.data_ptr())
            kdist.merge_top1_(top1)
            torch.cuda.synchronize(dev)
        node, tot = engine.decode_top1(top1.cpu().numpy().view(np.uint64))
        eng.close()
        m, f, l = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
        t_ref = np.where(m, f.astype(np.int64) + l, -1)
        want = np.where(t_ref.max(axis=1) >= 0, t_ref.argmax(axis=1), -1)
        q.put((rank, np.array_equal(got_n, ref_n) and np.array_equal(got_s, ref_s), np.array_equal(node, want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_engine_two_ranks_one_gpu():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, placed_ok, top1_ok in res:
        assert placed_ok, f"rank {rank}: sharded placement differs from the sequential oracle"
        assert top1_ok, f"rank {rank}: merged top-1 differs from the oracle"


def _gpu_rsv_worker(rank, world, port, q):
    from oracle import oracle

    _init(rank, world, port)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        cl = synth.make_rsv_cluster(5_000, 300, seed=72, n_quotas=15, quota_ratio=0.6, quota_tree=True)
        cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"),
                              eq_check_parent_quota=1)
        idx = np.arange(300)
        nodes = engine.build_node_rows(cfg, cl)
        pods = engine.build_pod_rows(cfg, cl, idx)
        got_n, got_s = kdist.place(cfg, nodes, pods, cl.now_ns, device=dev, reservations=cl.rsv_arr,
                                   quotas=cl.quota_arr)
        ref_n, ref_s, _, _ = oracle.schedule2(cfg, cl, idx, cl.now_ns)
        q.put((rank, np.array_equal(got_n, ref_n) and np.array_equal(got_s, ref_s), bool((ref_n == -1).any())))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_placement_reservation_quota_two_ranks_one_gpu():
    """Config 5 through the node-sharded placement: replicated reservation / quota state (a quota tree
    with EnableCheckParentQuota), per-tile partial keys merged over the ranks, identical resolves."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_rsv_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, placed_ok, some_rejected in res:
        assert placed_ok, f"rank {rank}: sharded placement differs from the sequential oracle"
        assert some_rejected


def _gpu_more_worker(rank, world, port, q, case):
    from oracle import oracle

    _init(rank, world, port)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        if case == "numa":
            # config 3 (NodeNUMAResource) through the node-sharded placement: zone commits in the resolve
            cl = synth.make_numa_cluster(3_000, 120, seed=73)
            cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "NodeNUMAResource"))
            idx = np.arange(120)
            nodes = engine.build_node_rows(cfg, cl)
            pods = engine.build_pod_rows(cfg, cl, idx)
            got_n, got_s = kdist.place(cfg, nodes, pods, cl.now_ns, device=dev)
            ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
            ok = np.array_equal(got_n, ref_n) and np.array_equal(got_s, ref_s)
        else:
            # Reservation + ElasticQuota matrix mode on each rank's shard, top-1 merged over the ranks
            cl = synth.make_rsv_cluster(3_000, 64, seed=74, rsv_node_frac=0.3, n_quotas=6, quota_ratio=0.4)
            cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"))
            idx = np.arange(64)
            nodes = engine.build_node_rows(cfg, cl)
            pods = engine.build_pod_rows(cfg, cl, idx)
            eng = kdist.sharded_engine(cfg, nodes, pods, dev, reservations=cl.rsv_arr, quotas=cl.quota_arr)
            with torch.cuda.stream(eng.torch_stream):
                top1 = torch.zeros(len(idx), dtype=torch.int64, device=dev)
                eng.eval_device(cl.now_ns, 0, 0, top1.data_ptr())
                kdist.merge_top1_(top1)
                torch.cuda.synchronize(dev)
            eng.close()
            ref = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)[5]
            ok = np.array_equal(top1.cpu().numpy().view(np.uint64), ref) and bool((ref > 0).any())
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["numa", "rsv_matrix"])
def test_sharded_more_two_ranks_one_gpu(case):
    """NodeNUMAResource placement and Reservation matrix mode through the two-rank sharded paths."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_more_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok, f"rank {rank}: {case} differs from the oracle"


def _gpu_config4_worker(rank, world, port, q, p_top, p_place):
    _init(rank, world, port)
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        c = synth.CONFIGS[4]
        cl = synth.make_cluster(c["n_nodes"], p_place, seed=c["seed"])
        cfg = shipped_profile()
        nodes = engine.build_node_rows(cfg, cl)
        pods = engine.build_pod_rows(cfg, cl, np.arange(p_place))
        eng = kdist.sharded_engine(cfg, nodes, pods[:p_top], dev)
        assert eng.shard == kdist.shard_range(len(nodes), rank, world)
        with torch.cuda.stream(eng.torch_stream):
            top1 = torch.zeros(p_top, dtype=torch.int64, device=dev)
            eng.eval_device(cl.now_ns, 0, 0, top1.data_ptr())
            kdist.merge_top1_(top1)
            torch.cuda.synchronize(dev)
        keys = top1.cpu().numpy().view(np.uint64).copy()
        eng.set_pods(pods)
        got_n, got_s = kdist.place_sharded(eng, cl.now_ns, dev, chunk=kdist.place_chunk_of(cfg))
        eng.close()
        q.put((rank, eng.shard, keys, got_n, got_s))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_config4_eight_ranks_gloo_rehearsal():
    """BASELINE config 4 (1M nodes, 8 shards of 125k) rehearsed with 8 gloo ranks sharing cuda:0: the
    merged top-1 of a 64-pod sample and the node-sharded placement of the first 128 pods (replicated
    snapshot, per-tile partial keys merged over the 8 ranks, identical resolves) against the oracle.
    RCCL over xGMI is the same protocol on 8 GPUs; that run is the driver's, unmeasured here."""
    from oracle import oracle

    world, p_top, p_place = 8, 64, 128
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_config4_worker, args=(r, world, port, q, p_top, p_place)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = synth.CONFIGS[4]
    cl = synth.make_cluster(c["n_nodes"], p_place, seed=c["seed"])
    cfg = shipped_profile()
    want_keys = oracle.eval_parallel(cfg, cl, np.arange(p_top), cl.now_ns, 16)
    ref_n, ref_s = oracle.schedule_parallel(cfg, cl, np.arange(p_place), cl.now_ns, 16)
    shards = sorted(r[1] for r in res)
    assert shards[0][0] == 0 and shards[-1][1] == c["n_nodes"] and all(b - a == 125_952 or b == c["n_nodes"]
                                                                        for a, b in shards[:-1])
    for rank, _, keys, got_n, got_s in res:
        np.testing.assert_array_equal(keys, want_keys, err_msg=f"rank {rank}: merged top-1")
        np.testing.assert_array_equal(got_n, ref_n, err_msg=f"rank {rank}: sharded placement")
        np.testing.assert_array_equal(got_s, ref_s, err_msg=f"rank {rank}: sharded placement scores")
    # the best nodes of the sample come from several shards
    owners = {int(n) // 125_952 for n in engine.decode_top1(want_keys)[0] if n >= 0}
    assert len(owners) >= 4


@pytest.mark.gpu
def test_bench_spawns_ranks_for_gpus_flag():
    """`python bench.py --gpus 8` without a launcher starts 8 ranks itself (gloo rehearsal on one GPU:
    matrix mode on node shards with the top-1 merge, then the node-sharded placement)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(HERE)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--backend", "gloo",
                          "--pods", "256", "--nodes", "20000", "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                          "--c3-pods", "0", "--c5-pods", "0"], capture_output=True, text=True, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-4000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["config"]["nodes_per_gpu"] == 2500
    assert line["placement"]["mode"].startswith("dist.place_sharded over 8 ranks")
    assert line["placement"]["placed"] > 200


def test_bench_rejects_mismatched_world():
    """--gpus must match WORLD_SIZE under a launcher; nccl cannot put more ranks than GPUs on a node."""
    import subprocess
    import sys

    root = os.path.dirname(HERE)
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, cwd=root, env=env)
    assert r.returncode == 2 and "must agree" in r.stderr
    if torch.cuda.device_count() < 64:
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "64"], capture_output=True,
                           text=True, timeout=300, cwd=root, env=env)
        assert r.returncode == 2 and "needs 64 GPUs" in r.stderr
