"""Placement parity at the sizes the bench times (SURVEY §8d gate 2), on the bench's own seeded clusters.

* config 1 exactly — seed 1, 1k pods × 5k nodes: every plane of every pair, and the whole placement
  against the oracle's sequential cycle, node rows afterwards against a host replay;
* config 2 — kg_place of all 10k pods over 100k nodes (seed 2) against the oracle's Parallelizer-faithful
  cycle (98 tiles, every top-16 list exhausted many times over, slow nodes crossing bounds mid-run), node
  rows afterwards against a host replay of the Reserve deltas;
* config 3 — NodeNUMAResource: a 32-pod plane sample of the 10k-pod matrix run (the pod-grouping
  permutation of kg_pods_set depends on the batch), and kg_place of all 1,000 bench pods at 100k nodes
  (the first 256 against the live oracle, all against the fixture);
* config 5 — a 100k-node seed-5 variant whose quota and allocate-once rejections start inside a
  1.5k-pod prefix, checked pod by pod against the oracle; and the bench's full 100k-pod burst: the first
  3k placements against the live oracle, every placement and the reservation / quota states after the
  burst against the fixture, plus invariants (no quota group or ancestor above its runtime or min, no
  reservation above its allocatable, reservation and quota deltas equal to what the placed pods request,
  rows equal the replay).

The live oracle runs on WORKERS host threads (ctypes releases the GIL).  The fixture
(tests/golden/fullsize_placements.npz, made by tests/golden/make_fullsize_placements.py — the same oracle
over the whole bursts, ≈ 35 min of host time) carries a digest of the engine inputs it was computed from;
a stale one fails the test rather than being compared.
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile
from oracle import oracle

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
import make_fullsize_placements as fullsize  # noqa: E402

pytestmark = pytest.mark.gpu

WORKERS = min(16, os.cpu_count() or 1)
RSV_EQ = ("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota")


def _replay(cfg, cl, idx, nodes):
    """Node rows after committing pod idx[p] to nodes[p] on the host (kg_row_commit, in queue order)."""
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes.tolist()):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    return rows


def _rows_by_pod_chunks(fn, P, parts=64):
    """fn(pod index array) → tuple of [k][N] planes over pod chunks in threads; rows stacked."""
    chunks = np.array_split(np.arange(P), min(parts, P))
    with ThreadPoolExecutor(WORKERS) as ex:
        outs = list(ex.map(fn, chunks))
    return [np.concatenate([o[i] for o in outs]) for i in range(len(outs[0]))]


def test_config1_exact_matrix_and_placement():
    c = synth.CONFIGS[1]
    P, N = c["n_pods"], c["n_nodes"]
    cl = synth.make_cluster(N, P, seed=c["seed"])
    cfg = shipped_profile()
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        res = eng.eval(cl.now_ns)
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    m, fit, la = _rows_by_pod_chunks(lambda i: oracle.eval_matrix(cfg, cl, i, cl.now_ns), P)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], fit)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], la)
    tot = np.where(m, fit.astype(np.int64) + la.astype(np.int64), -1)
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))
    ref_nodes, ref_scores = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))


def test_config2_full_placement():
    c = synth.CONFIGS[2]
    P, N = c["n_pods"], c["n_nodes"]
    cl = synth.make_cluster(N, P, seed=c["seed"])
    cfg = shipped_profile()
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_nodes, ref_scores = oracle.schedule_parallel(cfg, cl, idx, cl.now_ns, WORKERS)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    assert (nodes >= 0).mean() > 0.99
    # pods pile onto the best nodes: many nodes take several pods of the run
    assert np.bincount(nodes[nodes >= 0]).max() > 1
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))


def _numa_cfg():
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    return cfg


def test_config3_large_batch_plane_sample():
    P, N = 10_000, 100_000
    cl = synth.make_numa_cluster(N, P, seed=3)
    cfg = _numa_cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
        res = eng.eval(cl.now_ns)
    # every pod through its raw-spec group, then a direct sample
    from test_fullsize_gpu import _oracle_rows, check_planes_by_group, spec_groups
    check_planes_by_group(spec_groups(cl, P),
                          lambda reps: _oracle_rows(lambda i: oracle.eval_matrix3(cfg, cl, i, cl.now_ns), reps), res, N,
                          [lambda r, q: r["scores"][q, :, 0], lambda r, q: r["scores"][q, :, 1],
                           lambda r, q: r["numa_scores"][q]])
    pods = np.sort(np.random.default_rng(313).choice(P, 32, replace=False))
    with ThreadPoolExecutor(WORKERS) as ex:
        parts = list(ex.map(lambda p: oracle.eval_matrix3(cfg, cl, np.array([p]), cl.now_ns), pods))
    m, f, l, n = (np.concatenate([p[i] for p in parts]) for i in range(4))
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"][pods], N), m)
    np.testing.assert_array_equal(res["scores"][pods, :N, 0], f)
    np.testing.assert_array_equal(res["scores"][pods, :N, 1], l)
    np.testing.assert_array_equal(res["numa_scores"][pods, :N], n)
    tot = np.where(m, f.astype(np.int64) + l.astype(np.int64) + int(cfg["weight_numa"]) * n.astype(np.int64), -1)
    node, best = engine.decode_top1(res["top1"][pods])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))


def _fixture(key, dig):
    """The fixture's arrays of one case, after checking they were computed from these inputs."""
    fx = np.load(fullsize.OUT)
    assert str(fx[f"{key}_digest"]) == dig, f"{fullsize.OUT} is stale: rerun tests/golden/make_fullsize_placements.py"
    return fx


def test_config3_bench_placement():
    """kg_place of the bench's 1,000 NodeNUMAResource pods (pipelined chunks, the default with NUMA): the first
    256 against the live oracle, all 1,000 against the fixture, node rows against the replay."""
    cfg, cl, nrows, prows = fullsize.c3_case()
    P, K = len(prows), 256
    dig = fullsize.c3_digest(nrows, prows)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(nrows)
        eng.set_pods(prows)
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_nodes, ref_scores = oracle.schedule_parallel(cfg, cl, np.arange(K), cl.now_ns, WORKERS)
    np.testing.assert_array_equal(nodes[:K], ref_nodes)
    np.testing.assert_array_equal(scores[:K], ref_scores)
    fx = _fixture("c3", dig)
    np.testing.assert_array_equal(fx["c3_nodes"][:K], ref_nodes)   # the fixture agrees with the live oracle
    np.testing.assert_array_equal(nodes, fx["c3_nodes"])
    np.testing.assert_array_equal(scores, fx["c3_scores"])
    np.testing.assert_array_equal(after, _replay(cfg, cl, np.arange(P), nodes))


def _quota_invariants(q_after, q0):
    """No group above its runtime (used ≤ used_limit) or, for non-preemptible usage, above its min, on
    every resource the group limits; usage never shrinks."""
    for g in range(len(q_after)):
        lim_p, min_p = int(q_after["used_limit"]["present"][g]), int(q_after["min"]["present"][g])
        for r in range(nat.NUM_RES):
            u, nu = q_after["used"]["v"][g, r], q_after["non_preemptible_used"]["v"][g, r]
            assert u >= q0["used"]["v"][g, r]
            if (lim_p >> r) & 1:
                assert u <= q_after["used_limit"]["v"][g, r], (g, r)
            if (min_p >> r) & 1:
                assert nu <= q_after["min"]["v"][g, r], (g, r)


def test_config5_rejections_inside_checked_prefix():
    """Seed-5 variant: few reservation nodes (so allocate-once reservations run out), half of the owned
    pods requiring a matching reservation, quota runtimes at 60 % of demand — rejections of every kind
    start well inside the 1.5k-pod prefix that is checked pod by pod."""
    N, P = 100_000, 1_500
    cl = synth.make_rsv_cluster(N, P, seed=5, rsv_node_frac=0.004, quota_ratio=0.6, affinity_frac=0.5)
    cfg = shipped_profile(plugins=RSV_EQ)
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
        rsv_after = eng.download_reservations()
        q_after = eng.download_quotas()
    ref_nodes, ref_scores, ref_rsv, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    rejected = np.flatnonzero(ref_nodes < 0)
    assert len(rejected) > 50 and rejected[0] < 1_000
    once = (cl.rsv_arr["flags"] & nat.RSV_ALLOCATE_ONCE) != 0
    assert ((ref_rsv["n_assigned"] > cl.rsv_arr["n_assigned"]) & once).sum() >= 3   # allocate-once used up
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(rsv_after["n_assigned"], ref_rsv["n_assigned"])
    np.testing.assert_array_equal(rsv_after["allocated"]["v"], ref_rsv["allocated"]["v"])
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    np.testing.assert_array_equal(q_after["non_preemptible_used"]["v"], ref_q["non_preemptible_used"]["v"])
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))


def test_config5_full_burst():
    """The bench's own burst (100k batch pods × 100k nodes, seed 5) end to end: the first 3k placements against
    the oracle's cycle on WORKERS threads (kgo_schedule2_parallel), all 100k and the reservation and quota
    states after the burst against the fixture, then invariants over the whole run."""
    cfg, cl, nrows, prow = fullsize.c5_case()
    N, P = len(nrows), len(prow)
    idx = np.arange(P)
    dig = fullsize.c5_digest(cl, nrows, prow)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(nrows)
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(prow)
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
        rsv_after = eng.download_reservations()
        q_after = eng.download_quotas()
    placed = nodes >= 0
    assert 0.5 < placed.mean() < 0.95                      # the quota runtimes reject part of the burst
    K = 3_000
    ref_nodes, ref_scores, _, _ = oracle.schedule2(cfg, cl, idx[:K], cl.now_ns, workers=WORKERS)
    np.testing.assert_array_equal(nodes[:K], ref_nodes)
    np.testing.assert_array_equal(scores[:K], ref_scores)
    fx = _fixture("c5", dig)
    np.testing.assert_array_equal(fx["c5_nodes"][:K], ref_nodes)   # the fixture agrees with the live oracle
    np.testing.assert_array_equal(nodes, fx["c5_nodes"])
    np.testing.assert_array_equal(scores, fx["c5_scores"])
    np.testing.assert_array_equal(rsv_after["n_assigned"], fx["c5_rsv_n_assigned"])
    np.testing.assert_array_equal(rsv_after["allocated"]["v"], fx["c5_rsv_allocated"])
    np.testing.assert_array_equal(q_after["used"]["v"], fx["c5_quota_used"])
    np.testing.assert_array_equal(q_after["non_preemptible_used"]["v"], fx["c5_quota_np_used"])
    _quota_invariants(q_after, cl.quota_arr)
    # quota usage = Σ requests of the placed pods of each group (ElasticQuota.Reserve, plugin.go:323-337)
    q = cl.pods["quota"][:P]
    for r in (nat.RES_BATCH_CPU, nat.RES_BATCH_MEMORY):
        want = np.bincount(q[placed], weights=prow["request"][placed, r].astype(np.float64),
                           minlength=len(q_after)).astype(np.int64)
        np.testing.assert_array_equal(q_after["used"]["v"][:, r] - cl.quota_arr["used"]["v"][:, r], want)
    # reservations: a Restricted one never beyond its allocatable (Default / Aligned pods may also use the
    # node's free room, plugin.go:396-414); new assignments only on nodes that received pods
    restricted = rsv_after["policy"] == nat.RSV_POLICY_RESTRICTED
    assert restricted.any()
    assert (rsv_after["allocated"]["v"][restricted] <= rsv_after["allocatable"]["v"][restricted]).all()
    grew = rsv_after["n_assigned"] > cl.rsv_arr["n_assigned"]
    assert grew.any() and np.isin(rsv_after["node"][grew], nodes[placed]).all()
    once = (cl.rsv_arr["flags"] & nat.RSV_ALLOCATE_ONCE) != 0
    assert (rsv_after["n_assigned"][once] - cl.rsv_arr["n_assigned"][once] <= 1).all()
    # the reservation-held bytes that grew on a node are covered by the requests placed on it
    for r in (nat.RES_BATCH_CPU, nat.RES_BATCH_MEMORY):
        d_rsv = np.bincount(rsv_after["node"], weights=(rsv_after["allocated"]["v"][:, r] -
                                                        cl.rsv_arr["allocated"]["v"][:, r]).astype(np.float64),
                            minlength=N)
        d_pod = np.bincount(nodes[placed], weights=prow["request"][placed, r].astype(np.float64), minlength=N)
        assert (d_rsv <= d_pod).all()
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))
