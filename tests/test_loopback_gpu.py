"""kg_place_sharded at world 2 and 8 on ONE GPU: every rank is a process with its own engine, its own node shard
(kg_set_shard, shards above node 0 included) and the loopback communicator (kg_comm_init_loopback: the partial keys
merged through host shared memory instead of RCCL, which refuses two ranks on one device).  The chunk loop, the
per-chunk merges, the replicated resolve and the host Reserve are kg_place_sharded's own C++ — the code the driver's
2–8-GPU runs execute over RCCL, with only the merge transport swapped.  Placements and scores against the oracle's
sequential cycle for Fit + LoadAware (sequential and pipelined loops), NodeNUMAResource (pipelined, shard-local outcome
cache with its column offset), Reservation + ElasticQuota and cpuset batches (the host Reserve replicated); and the
failure contract: a rank that cannot set up makes every rank return an error, none hangs."""
import multiprocessing as mp
import os
import queue
import time
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _case(kind):
    from koordinator_amd import _native as nat
    from koordinator_amd import engine, synth
    from koordinator_amd.config import shipped_profile
    P = 240
    kw, forms, view, extra = {}, 0, None, {}
    if kind in ("fit_la", "fit_la_pipe"):
        cl = synth.make_cluster(8_192, P, seed=83)
        cfg = shipped_profile(place_chunk=16, fit_strategy="MostAllocated") if kind == "fit_la_pipe" else shipped_profile()
        forms = nat.FORM_PLACE_PIPELINE if kind == "fit_la_pipe" else 0
    elif kind == "numa":
        cl = synth.make_numa_cluster(8_192, P, seed=84)
        cfg = shipped_profile()
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    elif kind == "rsv_quota":
        from rsv_cases import rsv_cluster
        cl = rsv_cluster(8_192, P, seed=85, n_quotas=8, quota_ratio=0.6)
        cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"))
        kw = dict(reservations=cl.rsv_arr, quotas=cl.quota_arr)
    elif kind in ("cpuset", "cpuset_missing_table"):
        from bind_cases import make_bind_cluster
        cl, view, idx = make_bind_cluster(2_100, 160, 21, numa_frac=0.35)
        cfg = shipped_profile(place_chunk=16)
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
        extra = dict(idx=np.asarray(idx))
    else:
        raise ValueError(kind)
    src = view if view is not None else cl
    idx = extra.get("idx", np.arange(P))
    rows = engine.build_node_rows(cfg, src)
    pods = engine.build_pod_rows(cfg, src, idx)
    return cl, view, cfg, rows, pods, idx, kw, forms


def _worker(kind, rank, world, name, q):
    try:
        import torch
        from koordinator_amd import dist as kdist
        cl, view, cfg, rows, pods, idx, kw, forms = _case(kind)
        dev = torch.device("cuda", 0)
        eng = kdist.native_engine(cfg, rows, pods, dev, comm="loopback", rank=rank, world=world, shm_name=name, **kw)
        try:
            assert eng.comm_kind() == "loopback"
            if forms:
                eng.set_forms(forms)
            if view is not None and not (kind == "cpuset_missing_table" and rank == world - 1):
                eng.set_cpus(view)
            t0 = time.perf_counter()
            try:
                nodes, scores = eng.place_sharded(cl.now_ns)
            except Exception as ex:  # noqa: BLE001
                q.put((rank, ("error", str(ex), time.perf_counter() - t0)))
                return
            cpus = None
            if view is not None:
                from reserve_cycle import cpu_tables
                cpus = view.cpu_arr.copy()
                for j, (first, n, _, _) in cpu_tables(view).items():
                    cpus[first:first + n] = eng.download_cpus(j, n)
            q.put((rank, ("ok", nodes, scores, cpus, eng.download())))
        finally:
            eng.close()
    except Exception as ex:  # noqa: BLE001
        import traceback
        q.put((rank, ("crash", traceback.format_exc())))


def _run(kind, world, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/kg_lbtest_{os.getpid()}_{uuid.uuid4().hex[:8]}"
    ps = [ctx.Process(target=_worker, args=(kind, r, world, name, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    deadline = time.time() + timeout
    try:
        while len(out) < world and time.time() < deadline:
            try:
                r, v = q.get(timeout=2.0)
                out[r] = v
            except queue.Empty:
                if all(not p.is_alive() for p in ps) and q.empty():
                    break
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    assert len(out) == world, f"ranks answered: {sorted(out)} of {world} ({[p.exitcode for p in ps]})"
    return out


@pytest.mark.parametrize("kind,world", [("fit_la", 2), ("fit_la", 8), ("fit_la_pipe", 2), ("numa", 2), ("numa", 8),
                                        ("rsv_quota", 2), ("rsv_quota", 8), ("cpuset", 2)])
def test_place_sharded_loopback(kind, world):
    from oracle import oracle
    out = _run(kind, world)
    for r, v in out.items():
        assert v[0] == "ok", (r, v)
    cl, view, cfg, rows, pods, idx, kw, forms = _case(kind)
    if kind == "rsv_quota":
        ref_n, ref_s, _, _ = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    elif view is not None:
        ref_n, ref_s, ref_cpus = oracle.schedule_cpus(cfg, view, idx, cl.now_ns)
    else:
        ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    assert (ref_n >= 0).sum() > len(ref_n) // 2
    for r in range(world):
        _, nodes, scores, cpus, after = out[r]
        np.testing.assert_array_equal(nodes, ref_n, err_msg=f"rank {r}")
        np.testing.assert_array_equal(scores, ref_s, err_msg=f"rank {r}")
        np.testing.assert_array_equal(after, out[0][4], err_msg=f"rank {r}: replica rows differ")
        if view is not None:
            np.testing.assert_array_equal(cpus, ref_cpus, err_msg=f"rank {r}: CPUs")
    # the placements really span the shards: pods landed on nodes of more than one rank's shard
    from koordinator_amd.dist import shard_range
    owners = {next(k for k in range(world) if shard_range(len(rows), k, world)[0] <= n < shard_range(len(rows), k, world)[1])
              for n in ref_n[ref_n >= 0].tolist()}
    assert len(owners) > 1, owners


def test_place_sharded_loopback_setup_failure():
    """The last rank lacks the CPU tables a cpuset Reserve needs (bind_ready fails before the loop): it returns its
    own error, the others KG_ERR_STATE from the agreement, and nobody waits for a merge that never comes."""
    out = _run("cpuset_missing_table", 2, timeout=120)
    assert out[1][0] == "error" and "kg_cpus_set" in out[1][1], out[1]
    assert out[0][0] == "error" and "peer rank failed to set up" in out[0][1], out[0]
    assert out[0][2] < 60, out[0]
