"""LoadAwareScheduling resourceWeights beyond cpu / memory on the HIP engine vs the oracle: matrix mode
(k_eval_exact: every node on the exact int64 pair path), node shards, placement (the resolve re-scores
every node exactly), NodeNUMAResource and Reservation profiles (their kernels take kg_pair_exact on
such nodes)."""
import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu

W = {"cpu": 1, "memory": 1, "ephemeral-storage": 1, "example.com/gpu": 2, "kubernetes.io/batch-cpu": 1}
SF = {"ephemeral-storage": 60, "example.com/gpu": 100}


def _engine(cfg, view, idx):
    eng = engine.Engine(cfg)
    eng.load_snapshot(engine.build_node_rows(cfg, view))
    eng.set_pods(engine.build_pod_rows(cfg, view, idx))
    return eng


@pytest.mark.parametrize("shipped", [False, True], ids=["default", "shipped"])
def test_la_extra_matrix_parity(shipped):
    cl = synth.make_la_extra_cluster(2_600, 40, seed=41)
    kw = dict(resource_weights=W, estimated_scaling_factors=SF)
    cfg = shipped_profile(**kw) if shipped else make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling"), **kw)
    N, idx = len(cl.nodes), np.arange(40)
    with _engine(cfg, cl, idx) as eng:
        res = eng.eval(cl.now_ns)
    m, f, l = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], f)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], l)
    tot = np.where(m, int(cfg["weight_fit"]) * f.astype(np.int64) + int(cfg["weight_loadaware"]) * l, -1)
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))
    assert m.any()


def test_la_extra_matrix_equivalent_pods():
    """Pod equivalence on the exact path: 600 pods over 40 distinct rows, evaluated once per row."""
    cl = synth.make_la_extra_cluster(2_600, 40, seed=44)
    cfg = shipped_profile(resource_weights=W, estimated_scaling_factors=SF)
    N = len(cl.nodes)
    idx = np.random.default_rng(44).integers(0, 40, 600)
    with _engine(cfg, cl, idx) as eng:
        res = eng.eval(cl.now_ns)
    u, inv = np.unique(idx, return_inverse=True)
    m, f, l = oracle.eval_matrix(cfg, cl, u, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m[inv])
    np.testing.assert_array_equal(res["scores"][:, :N, 0], f[inv])
    np.testing.assert_array_equal(res["scores"][:, :N, 1], l[inv])
    tot = np.where(m, int(cfg["weight_fit"]) * f.astype(np.int64) + int(cfg["weight_loadaware"]) * l, -1)[inv]
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))


def test_la_extra_matrix_shard():
    cl = synth.make_la_extra_cluster(2_500, 24, seed=42)
    cfg = make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling"), resource_weights=W,
                      estimated_scaling_factors=SF)
    idx = np.arange(24)
    with _engine(cfg, cl, idx) as eng:
        eng.set_shard(1024, 2500)
        res = eng.eval(cl.now_ns)
    m, f, l = oracle.eval_matrix_range(cfg, cl, idx, 1024, 2500, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], 1476), m)
    np.testing.assert_array_equal(res["scores"][:, :1476, 1], l)


@pytest.mark.parametrize("chunk", [1, 16])
def test_la_extra_placement_matches_sequential_cycle(chunk):
    cl = synth.make_la_extra_cluster(1_200, 120, seed=43)
    cfg = shipped_profile(resource_weights=W, estimated_scaling_factors=SF, place_chunk=chunk)
    idx = np.arange(120)
    with _engine(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_nodes, ref_scores = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    np.testing.assert_array_equal(after["la_used_x"], rows["la_used_x"])
    assert (after["la_used_x"] != engine.build_node_rows(cfg, cl)["la_used_x"]).any()


def test_la_extra_with_numa_and_reservations():
    """The shipped profile's other engine plugins on top: NodeNUMAResource (k_eval_numa2 takes
    kg_pair_exact on every node) and Reservation + ElasticQuota (kg_rsv_pair)."""
    cl = synth.make_profile_cluster(1_500, 48, seed=44, rsv_node_frac=0.25, n_quotas=6, quota_ratio=0.3)
    plugins = ("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota", "NodeNUMAResource")
    cfg = shipped_profile(plugins=plugins, weight_numa=2, resource_weights={"cpu": 1, "memory": 1,
                                                                            "kubernetes.io/batch-cpu": 2})
    idx = np.arange(48)
    eng = engine.Engine(cfg)
    try:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        res = eng.eval(cl.now_ns)
    finally:
        eng.close()
    N = len(cl.nodes)
    m, fit, la, numa, rsv, top1 = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], la)
    np.testing.assert_array_equal(res["numa_scores"][:, :N], numa)
    np.testing.assert_array_equal(res["top1"], top1)
    assert nat.PLUGIN_NUMA & int(cfg["enabled_plugins"])


@pytest.mark.parametrize("shipped", [False, True], ids=["default", "shipped"])
def test_la_extra_fast_form_with_out_of_bound_nodes(shipped):
    """k_eval2's LAX form (the extra resources' fp64 planes): nodes whose extra-resource or native capacity lies
    outside the fp64 bounds (KGD_XSLOW) go to the exact pair path after it; planes and top-1 against the oracle,
    on a ragged node count and a shard."""
    cl = synth.make_la_extra_cluster(2_300, 48, seed=45)
    nodes = cl.nodes
    big = np.arange(7, 2_300, 61)
    nodes["allocatable"]["v"][big, nat.RES_EPHEMERAL_STORAGE] = (1 << 43) + 5
    huge = np.arange(11, 2_300, 97)
    nodes["allocatable"]["v"][huge, nat.RES_MEMORY] = (1 << 43) + 99
    cl = cl.with_nodes(nodes)
    kw = dict(resource_weights=W, estimated_scaling_factors=SF)
    cfg = shipped_profile(**kw) if shipped else make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling"), **kw)
    N, idx = len(cl.nodes), np.arange(48)
    with _engine(cfg, cl, idx) as eng:
        res = eng.eval(cl.now_ns)
        eng.set_shard(1024, 2300)
        shard = eng.eval(cl.now_ns)
    m, f, l = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], f)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], l)
    tot = np.where(m, int(cfg["weight_fit"]) * f.astype(np.int64) + int(cfg["weight_loadaware"]) * l, -1)
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))
    np.testing.assert_array_equal(engine.unpack_mask(shard["mask"], N - 1024), m[:, 1024:])
    np.testing.assert_array_equal(shard["scores"][:, :N - 1024, 1], l[:, 1024:])
    assert m[:, big].any()
