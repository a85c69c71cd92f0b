"""NodeNUMAResource (BASELINE config 3) on the HIP engine against the oracle restatement.

Matrix mode (k_eval_numa2: feasibility, Fit / LoadAware / NUMA score planes, top-1 keys), placement
(k_resolve with zone-allocation Reserve), node shards, and the host-side rejections of pods the
engine path does not cover (cpuset binding, more than two hint lists).
"""
import numpy as np
import pytest

from kat import load
from numa_cases import make_numa_edge_cluster, numa_config
from numa_kat import amplified_filter_cluster, amplified_score_cluster, numa_score_cluster
from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from oracle import oracle

pytestmark = pytest.mark.gpu

SCORE = load("numa_score_kat.json")
AMP = load("numa_amplified_kat.json")


def _engine_for(cfg, view, pod_index):
    eng = engine.Engine(cfg)
    eng.load_snapshot(engine.build_node_rows(cfg, view))
    eng.set_pods(engine.build_pod_rows(cfg, view, pod_index))
    return eng


def _weights(cfg):
    return int(cfg["weight_fit"]), int(cfg["weight_loadaware"]), int(cfg["weight_numa"])


def _check_matrix3(cfg, cl, P, begin=0, end=None, idx=None, forms=0):
    N = len(cl.nodes)
    end = N if end is None else end
    idx = np.arange(P) if idx is None else idx
    with _engine_for(cfg, cl, idx) as eng:
        eng.set_forms(forms)
        if (begin, end) != (0, N):
            eng.set_shard(begin, end)
        res = eng.eval(cl.now_ns)
    W = end - begin
    m, f, l, n = oracle.eval_matrix3(cfg, cl, idx, cl.now_ns, begin, end)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], W), m)
    np.testing.assert_array_equal(res["scores"][:, :W, 0], f)
    np.testing.assert_array_equal(res["scores"][:, :W, 1], l)
    np.testing.assert_array_equal(res["numa_scores"][:, :W], n)
    wf, wl, wn = _weights(cfg)
    tot = np.where(m, wf * f.astype(np.int64) + wl * l.astype(np.int64) + wn * n.astype(np.int64), -1)
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1) + begin, -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))
    return m


def test_matrix_config3_mix():
    cl = synth.make_numa_cluster(3_000, 48, seed=3)
    m = _check_matrix3(numa_config(), cl, 48)
    assert 0.2 < m.mean() < 0.95


@pytest.mark.parametrize("seed,kw", [(11, {}), (12, dict(numa_strategy="MostAllocated", weight_numa=3,
                                                           numa_hint_strategy="MostAllocated"))])
def test_matrix_numa_edge_cases(seed, kw):
    cl = make_numa_edge_cluster(2_100, 64, seed=seed)
    _check_matrix3(numa_config(**kw), cl, 64)


@pytest.mark.parametrize("seed,pods", [(14, 160), (15, 333)])
def test_matrix_numa_grouped_pods(seed, pods):
    # > 64 pods: k_eval_numa2 walks the batch in hint-list-grouped order (kg_pods_set's numa_perm) and
    # must still write every pod's own row
    cl = make_numa_edge_cluster(2_100, pods, seed=seed)
    _check_matrix3(numa_config(), cl, pods)
    cl3 = synth.make_numa_cluster(2_000, pods, seed=seed)
    _check_matrix3(numa_config(), cl3, pods)


@pytest.mark.parametrize("begin,end", [(0, None), (1024, 2300)])
def test_matrix_numa_equivalent_pods(begin, end):
    """Pod equivalence (kg_engine::eq_on): a batch of 700 pods over 120 distinct rows is evaluated as its distinct
    rows, whose output rows are copied to every pod of each; planes and top-1 against the oracle, also on a
    shard, and a device-output pass equal to the host-output one."""
    cl = make_numa_edge_cluster(2_300, 120, seed=51)
    idx = np.random.default_rng(51).integers(0, 120, 700)
    _check_matrix3(numa_config(), cl, len(idx), begin=begin, end=end, idx=idx)


def test_matrix_numa_equivalent_pods_device_outputs():
    import torch
    cl = synth.make_numa_cluster(2_000, 600, seed=52)
    cfg = numa_config()
    idx = np.arange(600)
    # torch's HIP context first (it does not initialise beside a live engine)
    dev = torch.device("cuda", 0)
    W = (len(cl.nodes) + 63) // 64
    mask = torch.zeros((600, W), dtype=torch.int64, device=dev)
    scores = torch.zeros((600, W * 64, 2), dtype=torch.uint8, device=dev)
    numa = torch.zeros((600, W * 64), dtype=torch.uint8, device=dev)
    top1 = torch.zeros(600, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    with _engine_for(cfg, cl, idx) as eng:
        host = eng.eval(cl.now_ns)
        assert eng.mask_words == W
        eng.eval_device(cl.now_ns, mask.data_ptr(), scores.data_ptr(), top1.data_ptr(), numa.data_ptr())
        eng.sync()
    np.testing.assert_array_equal(mask.cpu().numpy().view(np.uint64), host["mask"])
    np.testing.assert_array_equal(scores.cpu().numpy(), host["scores"])
    np.testing.assert_array_equal(numa.cpu().numpy(), host["numa_scores"])
    np.testing.assert_array_equal(top1.cpu().numpy().view(np.uint64), host["top1"])


def test_matrix_numa_shard():
    cl = make_numa_edge_cluster(2_500, 40, seed=13)
    _check_matrix3(numa_config(), cl, 40, begin=1024, end=2500)


def test_matrix_numa_huge_zone_memory():
    # zone memory totals of 2^42..2^48 bytes: the device's score quotients take one fp64 division up to a
    # divisor of 2^46 and the exact int64 division beyond (kg_qdiv), both against the oracle's int64 quotients
    cl = make_numa_edge_cluster(2_100, 64, seed=41)
    numa = cl.numa_arr
    for j in range(len(cl.nodes)):
        f = (1, 64, 1024)[j % 3]
        for z in range(int(numa["n_zones"][j])):
            numa["zone_total"][j, z]["v"][nat.RES_MEMORY] *= f
            numa["zone_allocated"][j, z]["v"][nat.RES_MEMORY] *= f
    assert (numa["zone_total"]["v"][:, :, nat.RES_MEMORY].astype(np.float64) >= 2.0 ** 46).any()
    _check_matrix3(numa_config(), cl, 64)


@pytest.mark.parametrize("pods,begin,end", [(40, 0, None), (333, 0, None), (97, 1024, 2500)])
def test_matrix_numa_queued_form(pods, begin, end):
    # KG_FORM_NUMA_QUEUED: k_eval_numa2's queued form (32-node work items from a device counter, half mask
    # words) on launches the size rule keeps on the grid form — the full-size launches take it by default
    _check_matrix3(numa_config(), make_numa_edge_cluster(2_500, pods, seed=21 + pods), pods, begin=begin, end=end,
                   forms=nat.FORM_NUMA_QUEUED)


@pytest.mark.parametrize("forms", [nat.FORM_NUMA_FUSED, nat.FORM_NUMA_FUSED | nat.FORM_NUMA_QUEUED, 0, nat.FORM_NUMA_QUEUED])
@pytest.mark.parametrize("pods,begin,end,dup", [(97, 0, None, False), (333, 1024, 2500, False), (700, 0, None, True)])
def test_matrix_numa_fused_and_combined(forms, pods, begin, end, dup):
    """The two matrix forms of NodeNUMAResource: Fit + LoadAware inside k_eval_numa2 (KG_FORM_NUMA_FUSED), and the
    default for launches with planes — the class / slot kernels' Fit + LoadAware pass, then k_eval_numa2 adding the
    NodeNUMAResource term to those planes (also over the distinct rows of an equivalent-pod batch, `dup`)."""
    cl = make_numa_edge_cluster(2_500, 120 if dup else pods, seed=61 + pods)
    idx = np.random.default_rng(61).integers(0, 120, pods) if dup else None
    _check_matrix3(numa_config(), cl, pods, begin=begin, end=end, idx=idx, forms=forms)


@pytest.mark.parametrize("case", SCORE["cases"], ids=lambda c: c["name"])
def test_kat_numa_node_score(case):
    """TestNUMANodeScore (nodenumaresource/scoring_test.go) through kg_eval."""
    cfg, view, pi, cl = numa_score_cluster(case)
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(0)
    k = len(case["nodes"])
    assert list(res["numa_scores"][0, :k]) == case["want"]
    assert engine.unpack_mask(res["mask"], k).all()


@pytest.mark.parametrize("case", AMP["score_cases"], ids=lambda c: c["name"])
def test_kat_amplified_score(case):
    """TestScoreWithAmplifiedCPUs through kg_eval, cpuset pods included (matrix mode)."""
    cfg, view, pi, cl = amplified_score_cluster(case)
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(0)
    k = len(case["nodes"])
    assert list(res["numa_scores"][0, :k]) == case["want"]
    assert engine.unpack_mask(res["mask"], k).all()


@pytest.mark.parametrize("case", AMP["filter_cases"], ids=lambda c: c["name"])
def test_kat_amplified_filter(case):
    """TestFilterWithAmplifiedCPUs through kg_eval (NodeNUMAResource alone)."""
    cfg, view, pi, cl = amplified_filter_cluster(case)
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(0)
    assert bool(engine.unpack_mask(res["mask"], 1)[0, 0]) == case["want"]


@pytest.mark.parametrize("chunk,numa2", [(1, False), (16, False), (64, False), (1, True), (16, True)])
def test_placement_numa_matches_sequential_cycle(chunk, numa2):
    cl = make_numa_edge_cluster(700, 200, seed=21)
    cfg = numa_config(weight_numa=2, place_chunk=chunk)
    idx = np.arange(200)
    with _engine_for(cfg, cl, idx) as eng:
        if numa2:   # every chunk through k_eval_numa2's queued form (one key per tile) instead of k_eval_numa_chunk
            eng.set_forms(nat.FORM_NUMA_CHUNK_TILE)
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    np.testing.assert_array_equal(after, rows)
    assert (after["zone_allocated"] != engine.build_node_rows(cfg, cl)["zone_allocated"]).any()


def test_placement_numa_tight_cluster():
    """Few NUMA nodes: zones fill up, SingleNUMANode / Restricted start rejecting, pods go unplaced."""
    cl = make_numa_edge_cluster(12, 400, seed=31)
    cfg = numa_config(place_chunk=32)
    idx = np.arange(400)
    with _engine_for(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    assert (ref_n == -1).any()
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)


def test_pods_set_rejects_numa_shapes_off_the_engine_path():
    cl = synth.make_numa_cluster(100, 4, seed=5)
    cfg = numa_config()
    rows = engine.build_pod_rows(cfg, cl, np.arange(4))
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        bad = rows.copy()
        bad["flags"][1] |= nat.POD_NUMA_CPU_BIND
        bad["flags"][1] &= ~np.uint32(nat.POD_NUMA_SKIP)
        eng.set_pods(bad)   # cpusets need the nodes' CPU detail (these zoned nodes have none): refused at evaluation
        with pytest.raises(engine.EngineError, match="cpuset"):
            eng.eval(cl.now_ns)
        bad = rows.copy()
        bad["flags"][2] &= ~np.uint32(nat.POD_NUMA_SKIP)
        bad["numa_request_present"][2] = 0b111   # cpu, memory and a zero-valued ephemeral-storage key
        bad["numa_request"][2, 2] = 0
        with pytest.raises(engine.EngineError, match="hint lists"):
            eng.set_pods(bad)
        eng.set_pods(rows)   # the batch itself is fine


@pytest.mark.parametrize("case", load("numa_plugin_score_kat.json")["cases"], ids=lambda c: c["name"])
def test_kat_plugin_score_gpu(case):
    """TestPlugin_Score (scoring_test.go:332-551): cpuset-pod node scores through kg_eval."""
    from test_numa_plugin_kat2 import score_cluster
    cfg, view, pi = score_cluster(case)
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(0)
    assert bool(engine.unpack_mask(res["mask"], 1)[0, 0])
    assert int(res["numa_scores"][0, 0]) == case["want"]


@pytest.mark.parametrize("case", load("numa_node_scoring_kat.json")["cases"], ids=lambda c: c["name"])
def test_kat_filter_with_numa_node_scoring_gpu(case):
    """TestFilterWithNUMANodeScoring (plugin_test.go:1649-1877): kg_commit allocates on the stored hint's zone."""
    from test_numa_plugin_kat2 import node_scoring_cluster
    cfg, view, pi = node_scoring_cluster(case)
    with _engine_for(cfg, view, [pi]) as eng:
        before = eng.download()["zone_allocated"][0].copy()
        assert eng.commit(0, 0)
        after = eng.download()["zone_allocated"][0]
    assert np.flatnonzero((after != before).any(axis=1)).tolist() == [case["want_zone"]]
