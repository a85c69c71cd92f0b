"""Reservation + ElasticQuota (config 5) on the HIP engine vs the oracle: matrix mode (mask, plugin
planes, normalized Reservation plane, top1) and placement (sequential cycle parity, reservation and
quota state after the last Reserve, snapshot rows)."""
import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle
from rsv_cases import filter_view, kat_cluster, kat_doc, order_view, restore_filter_doc, rsv_cluster

pytestmark = pytest.mark.gpu

RSV = ("NodeResourcesFit", "LoadAwareScheduling", "Reservation")
RSV_EQ = RSV + ("ElasticQuota",)
PROFILE = RSV_EQ + ("NodeNUMAResource",)   # the shipped profile's engine plugins


def _engine(cfg, view, idx):
    eng = engine.Engine(cfg)
    eng.load_snapshot(engine.build_node_rows(cfg, view))
    if int(cfg["enabled_plugins"]) & 0x8:
        eng.set_reservations(view.rsv_arr)
    if int(cfg["enabled_plugins"]) & 0x10:
        eng.set_quotas(view.quota_arr)
    eng.set_pods(engine.build_pod_rows(cfg, view, idx))
    return eng


def _check_matrix(cfg, cl, idx):
    N = len(cl.nodes)
    with _engine(cfg, cl, idx) as eng:
        res = eng.eval(cl.now_ns)
    m, fit, la, numa, rsv, top1 = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], fit)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], la)
    if int(cfg["enabled_plugins"]) & nat.PLUGIN_NUMA:
        np.testing.assert_array_equal(res["numa_scores"][:, :N], numa)
    np.testing.assert_array_equal(res["rsv_scores"][:, :N], rsv)
    np.testing.assert_array_equal(res["top1"], top1)
    return m, rsv


@pytest.mark.parametrize("case", kat_doc()["cases"], ids=lambda c: c["name"])
def test_reservation_score_kat_single_node(case):
    """TestScore KATs through kg_eval: on one node NormalizeScore maps any positive score to 100."""
    cfg = make_config(plugins=("Reservation",))
    view = kat_cluster(kat_doc(), case)
    with _engine(cfg, view, [0]) as eng:
        res = eng.eval(view.now_ns)
    assert int(res["rsv_scores"][0, 0]) == (100 if case["want"] > 0 else 0)


@pytest.mark.parametrize("plugins", [RSV, RSV_EQ], ids=["rsv", "rsv+quota"])
def test_rsv_matrix_parity(plugins):
    cl = rsv_cluster(3000, 80, seed=61, rsv_node_frac=0.2, n_quotas=8, quota_ratio=0.01)
    m, rsv = _check_matrix(shipped_profile(plugins=plugins), cl, np.arange(80))
    assert m.any() and rsv.max() == 100


def test_rsv_matrix_ragged_and_weights():
    cl = rsv_cluster(1537, 33, seed=62, rsv_node_frac=0.5)
    cfg = make_config(plugins=RSV, weight_fit=3, weight_loadaware=2, weight_reservation=7,
                      fit_strategy="MostAllocated")
    _check_matrix(cfg, cl, np.arange(33))


@pytest.mark.parametrize("chunk", [1, 16, 64])
def test_rsv_placement_matches_sequential_cycle(chunk):
    cl = rsv_cluster(3000, 400, seed=63, n_quotas=16, quota_ratio=0.6)
    cfg = shipped_profile(plugins=RSV_EQ, place_chunk=chunk)
    idx = np.arange(400)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
        rsv_after = eng.download_reservations()
        q_after = eng.download_quotas()
    ref_nodes, ref_scores, ref_rsv, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    assert (ref_nodes == -1).any() and (ref_nodes >= 0).any()
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    for f in ("n_assigned",):
        np.testing.assert_array_equal(rsv_after[f], ref_rsv[f])
    np.testing.assert_array_equal(rsv_after["allocated"]["v"], ref_rsv["allocated"]["v"])
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    np.testing.assert_array_equal(q_after["non_preemptible_used"]["v"], ref_q["non_preemptible_used"]["v"])
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    np.testing.assert_array_equal(after, rows)


def test_rsv_placement_tight_allocate_once():
    """Few nodes, every node with reservations: allocate-once reservations close after one pod,
    required-affinity pods run out of reservations, quota groups run dry."""
    cl = rsv_cluster(40, 600, seed=64, rsv_node_frac=1.0, n_quotas=3, quota_ratio=0.5, affinity_frac=0.5)
    cfg = shipped_profile(plugins=RSV_EQ, place_chunk=32)
    idx = np.arange(600)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        rsv_after = eng.download_reservations()
    ref_nodes, ref_scores, ref_rsv, _ = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(rsv_after["n_assigned"], ref_rsv["n_assigned"])


def test_rsv_commit_one():
    cl = rsv_cluster(500, 10, seed=65, rsv_node_frac=1.0)
    cfg = shipped_profile(plugins=RSV_EQ)
    with _engine(cfg, cl, np.arange(10)) as eng:
        _, _, ref_rsv, ref_q = oracle.schedule2(cfg, cl, np.arange(1), cl.now_ns)
        ref_nodes, _, _, _ = oracle.schedule2(cfg, cl, np.arange(1), cl.now_ns)
        if ref_nodes[0] >= 0:
            eng.commit(0, int(ref_nodes[0]))
            np.testing.assert_array_equal(eng.download_reservations()["allocated"]["v"], ref_rsv["allocated"]["v"])
            np.testing.assert_array_equal(eng.download_quotas()["used"]["v"], ref_q["used"]["v"])


def test_commit_needs_every_quota_group():
    """kg_commit checks that the pod's quota group exists (quota_ready), like kg_eval and kg_place do:
    a commit after kg_quota_set got fewer groups than the pods reference fails with KG_ERR_STATE."""
    cl = rsv_cluster(200, 8, seed=66, rsv_node_frac=1.0, n_quotas=3)
    cfg = shipped_profile(plugins=RSV_EQ)
    eng = engine.Engine(cfg)
    try:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr[:1])
        rows = engine.build_pod_rows(cfg, cl, np.arange(8))
        rows["quota"][:] = 2
        eng.set_pods(rows)
        with pytest.raises(engine.EngineError, match="quota index"):
            eng.commit(0, 0)
    finally:
        eng.close()


def test_profile_matrix_parity():
    """Every engine plugin of the shipped profile at once (Fit, LoadAware, NodeNUMAResource, Reservation,
    ElasticQuota): NUMA planes of reservation nodes come from the restored NodeInfo."""
    cl = synth.make_profile_cluster(2600, 72, seed=71, rsv_node_frac=0.25, n_quotas=8, quota_ratio=0.3)
    m, rsv = _check_matrix(shipped_profile(plugins=PROFILE, weight_numa=2), cl, np.arange(72))
    assert m.any() and rsv.max() == 100


@pytest.mark.parametrize("chunk", [1, 8, 64])
def test_profile_placement_matches_sequential_cycle(chunk):
    cl = synth.make_profile_cluster(900, 260, seed=72, rsv_node_frac=0.3, n_quotas=6, quota_ratio=0.5)
    cfg = shipped_profile(plugins=PROFILE, weight_numa=2, place_chunk=chunk)
    idx = np.arange(260)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        rsv_after = eng.download_reservations()
        q_after = eng.download_quotas()
        rows_after = eng.download()
    ref_nodes, ref_scores, ref_rsv, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(rsv_after["n_assigned"], ref_rsv["n_assigned"])
    np.testing.assert_array_equal(rsv_after["allocated"]["v"], ref_rsv["allocated"]["v"])
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    rnodes = set(cl.rsv_arr["node"].tolist())
    assert any(n in rnodes for n in nodes.tolist())
    assert (rows_after["zone_allocated"] != engine.build_node_rows(cfg, cl)["zone_allocated"]).any()


RF = restore_filter_doc()


@pytest.mark.parametrize("case", RF["filter"]["cases"], ids=lambda c: c["name"])
def test_filter_with_reservations_kat_gpu(case):
    """Test_filterWithReservations cases through kg_eval (Reservation alone)."""
    cfg = make_config(plugins=("Reservation",))
    view = filter_view(RF, case)
    with _engine(cfg, view, [0]) as eng:
        res = eng.eval(view.now_ns)
    assert bool(engine.unpack_mask(res["mask"], 1)[0, 0]) == case["want"]


def test_score_with_order_kat_gpu():
    """TestScoreWithOrder through kg_eval: normalized 10/10/10/100, best node test-node-4."""
    cfg = make_config(plugins=("Reservation",))
    view = order_view(RF)
    with _engine(cfg, view, [0]) as eng:
        res = eng.eval(view.now_ns)
    assert list(res["rsv_scores"][0, :4]) == RF["score_with_order"]["want"]
    assert engine.decode_top1(res["top1"])[0][0] == 3


@pytest.mark.parametrize("world", [2, 3])
def test_rsv_matrix_sharded(world):
    """Reservation matrix mode under node shards (the multi-GPU matrix path on one device): every shard
    evaluates all reservation nodes, writes only its own columns, and the max over the shards' top1
    keys (dist.merge_top1_) equals the unsharded result and the oracle's."""
    from koordinator_amd.dist import shard_range
    cl = synth.make_profile_cluster(2600, 48, seed=79, rsv_node_frac=0.3, n_quotas=6, quota_ratio=0.3)
    cfg = shipped_profile(plugins=PROFILE, weight_numa=2)
    N, idx = len(cl.nodes), np.arange(48)
    m, fit, la, numa, rsv, top1 = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    best = np.zeros(48, np.uint64)
    with _engine(cfg, cl, idx) as eng:
        for r in range(world):
            b, e = shard_range(N, r, world)
            eng.set_shard(b, e)
            res = eng.eval(cl.now_ns)
            W = e - b
            np.testing.assert_array_equal(engine.unpack_mask(res["mask"], W), m[:, b:e])
            np.testing.assert_array_equal(res["scores"][:, :W, 0], fit[:, b:e])
            np.testing.assert_array_equal(res["scores"][:, :W, 1], la[:, b:e])
            np.testing.assert_array_equal(res["numa_scores"][:, :W], numa[:, b:e])
            np.testing.assert_array_equal(res["rsv_scores"][:, :W], rsv[:, b:e])
            best = np.maximum(best, res["top1"].astype(np.uint64))
    np.testing.assert_array_equal(best, top1)
    assert rsv.max() == 100 and (top1 > 0).any()


def test_rsv_many_per_node_matrix_and_placement():
    """Up to 12 reservations per node: matrix planes and the sequential cycle vs the oracle."""
    cl = rsv_cluster(1500, 200, seed=78, rsv_node_frac=0.3, max_rsv_per_node=12)
    assert np.bincount(cl.rsv_arr["node"]).max() > 8
    cfg = shipped_profile(plugins=RSV_EQ)
    idx = np.arange(200)
    _check_matrix(cfg, cl, idx)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
    ref_nodes, ref_scores, _, _ = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)


@pytest.mark.parametrize("check_parent", [0, 1])
@pytest.mark.parametrize("chunk", [1, 16])
def test_quota_tree_placement_matches_sequential_cycle(check_parent, chunk):
    """A quota tree (binary heap of 15 groups): Reserve walks the ancestors, EnableCheckParentQuota gates
    on them (k_resolve's gate and commit); quota states after the cycle equal the oracle's."""
    cl = rsv_cluster(2000, 400, seed=67, n_quotas=15, quota_ratio=0.5, quota_tree=True)
    cfg = shipped_profile(plugins=RSV_EQ, place_chunk=chunk, eq_check_parent_quota=check_parent)
    idx = np.arange(400)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        q_after = eng.download_quotas()
    ref_nodes, ref_scores, _, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    assert (ref_nodes == -1).any() and (ref_nodes >= 0).any()
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    np.testing.assert_array_equal(q_after["non_preemptible_used"]["v"], ref_q["non_preemptible_used"]["v"])
    np.testing.assert_array_equal(q_after["parent"], cl.quota_arr["parent"])


def test_quota_tree_matrix_parent_gate():
    """Matrix mode (k_pod_gate) with ancestors already near their limits: the parent check closes pods
    whose own group has room."""
    cl = rsv_cluster(1500, 120, seed=68, n_quotas=7, quota_ratio=0.6, quota_tree=True)
    q = cl.quota_arr
    q["used"] = q["used_limit"]
    q["used"]["v"][1:] = 0
    q["used"]["v"][0] = np.maximum(q["used_limit"]["v"][0] - 1, 0)   # the root-most group is full
    off = _check_matrix(shipped_profile(plugins=RSV_EQ), cl, np.arange(120))[0]
    on = _check_matrix(shipped_profile(plugins=RSV_EQ, eq_check_parent_quota=1), cl, np.arange(120))[0]
    closed = off.any(axis=1) & ~on.any(axis=1)
    assert closed.any() and not (on & ~off).any()


def test_quota_set_rejects_cyclic_tree():
    cl = rsv_cluster(64, 4, seed=69, n_quotas=3, quota_tree=True)
    q = cl.quota_arr.copy()
    q["parent"] = [1, 2, 0]
    with engine.Engine(shipped_profile(plugins=RSV_EQ)) as eng:
        with pytest.raises(RuntimeError, match="cyclic"):
            eng.set_quotas(q)
        q["parent"] = [-1, 5, 0]
        with pytest.raises(RuntimeError, match="out of range"):
            eng.set_quotas(q)
        q["parent"] = 0          # a zero-filled record: group 0 its own parent
        with pytest.raises(RuntimeError, match="its own parent"):
            eng.set_quotas(q)
