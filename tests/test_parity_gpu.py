"""Parity of the HIP engine (through the C-ABI) against the CPU oracle and the reference KATs."""
import numpy as np
import pytest

from kat import case_cluster, load
from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu

DOC = load("loadaware_kat.json")


def _engine_for(cfg, view, pod_index):
    eng = engine.Engine(cfg)
    eng.load_snapshot(engine.build_node_rows(cfg, view))
    eng.set_pods(engine.build_pod_rows(cfg, view, pod_index))
    return eng


@pytest.mark.parametrize("case", DOC["score_cases"], ids=lambda c: c["name"])
def test_kat_loadaware_score(case):
    cfg, view, pi, cl = case_cluster(DOC, case, "pod")
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(cl.now_ns)
    assert int(res["scores"][0, 0, 1]) == case["want"]


@pytest.mark.parametrize("case", DOC["filter_cases"], ids=lambda c: c["name"])
def test_kat_loadaware_filter(case):
    cfg, view, pi, cl = case_cluster(DOC, case, "test_pod")
    cfg["enabled_plugins"] = 0x2  # LoadAwareScheduling only, like the reference test framework
    with _engine_for(cfg, view, [pi]) as eng:
        res = eng.eval(cl.now_ns)
    feasible = bool(res["mask"][0, 0] & np.uint64(1))
    assert feasible == (case["want"] == 0)


def _check_matrix(cfg, view, pod_index, now_ns):
    N = len(view.nodes)
    with _engine_for(cfg, view, pod_index) as eng:
        res = eng.eval(now_ns)
    m_ref, fit_ref, la_ref = oracle.eval_matrix(cfg, view, pod_index, now_ns)
    mask = engine.unpack_mask(res["mask"], N)
    np.testing.assert_array_equal(mask, m_ref)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], fit_ref)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], la_ref)
    total = int(cfg["weight_fit"]) * fit_ref.astype(np.int64) + int(cfg["weight_loadaware"]) * la_ref.astype(np.int64)
    total = np.where(m_ref, total, -1)
    best = total.argmax(axis=1)  # lowest index among ties
    node, tot = engine.decode_top1(res["top1"])
    want_node = np.where(total.max(axis=1) >= 0, best, -1)
    np.testing.assert_array_equal(node, want_node)
    np.testing.assert_array_equal(tot, total.max(axis=1))


@pytest.mark.parametrize("profile", ["default", "shipped", "most"])
def test_matrix_parity_config1_shape(profile):
    cl = synth.make_cluster(5_000, 96, seed=11)
    cfg = {"default": make_config, "shipped": shipped_profile,
           "most": lambda: make_config(fit_strategy="MostAllocated",
                                       fit_resources={"cpu": 2, "memory": 1, "kubernetes.io/batch-cpu": 3})}[profile]()
    _check_matrix(cfg, cl, np.arange(96), cl.now_ns)


@pytest.mark.parametrize("profile", ["least4", "most4", "w2"])
def test_matrix_parity_uniform_slot_fold(profile):
    """Batch pods score cpu / memory at the NonZero defaults (one value for the whole class): the class
    path folds those slots into a per-node term (kg_cls_desc::uni_res); it must equal the oracle under
    LeastAllocated / MostAllocated and non-unit weights."""
    four = ("cpu", "memory", "kubernetes.io/batch-cpu", "kubernetes.io/batch-memory")
    cfg = {"least4": lambda: make_config(fit_resources={r: 1 for r in four}),
           "most4": lambda: make_config(fit_strategy="MostAllocated", fit_resources={r: 1 for r in four}),
           "w2": lambda: make_config(fit_resources={r: 2 for r in four})}[profile]()
    cl = synth.make_cluster(3_000, 160, seed=21)
    _check_matrix(cfg, cl, np.arange(160), cl.now_ns)


def _distinct_rows(cl, n_pods, seed):
    """Every pending pod gets its own ephemeral-storage request (and every node room for it): the class rows
    are then pairwise distinct while the ~105 cpu / memory shapes still share EstimatePods."""
    rng = np.random.default_rng(seed)
    cont = cl.containers
    eph = rng.permutation(n_pods).astype(np.int64) * 4096 + (1 << 30)
    first = cl.pods["first_container"][:n_pods]
    cont["requests"]["v"][first, nat.RES_EPHEMERAL_STORAGE] = eph
    cont["requests"]["present"][first] |= np.uint32(1 << nat.RES_EPHEMERAL_STORAGE)
    nodes = cl.nodes
    nodes["allocatable"]["v"][:, nat.RES_EPHEMERAL_STORAGE] = rng.integers(1 << 30, 1 << 40, len(nodes))
    nodes["allocatable"]["present"] |= np.uint32(1 << nat.RES_EPHEMERAL_STORAGE)
    nodes["requested"]["v"][:, nat.RES_EPHEMERAL_STORAGE] = rng.integers(0, 1 << 39, len(nodes))
    return cl.with_nodes(nodes)


@pytest.mark.parametrize("profile", ["shipped", "default", "prod_usage", "most_w"])
def test_matrix_parity_la_uniform_chunks(profile):
    """k_eval3's plain part groups a class's pods by EstimatePod and evaluates the LoadAware sums of a whole
    chunk of one estimate once per node (kg_cls_desc::la_uni_end).  1,600 pods with pairwise distinct class
    rows (each its own ephemeral-storage request) over ~105 request shapes give both uniform chunks and a
    mixed tail per class; some nodes are beyond the fp64 bounds and the node count is ragged."""
    cfg = {"shipped": shipped_profile, "default": make_config,
           "prod_usage": lambda: shipped_profile(score_according_prod_usage=True),
           "most_w": lambda: make_config(fit_strategy="MostAllocated", fit_resources={"cpu": 2, "memory": 1})}[profile]()
    cl = synth.make_cluster(1_100, 1_600, seed=31)
    big = np.arange(3, 1_100, 97)
    cl.nodes["allocatable"]["v"][big, 1] = (1 << 43) + 99
    cl = _distinct_rows(cl.with_nodes(cl.nodes), 1_600, 31)
    _check_matrix(cfg, cl, np.arange(1_600), cl.now_ns)


def _dup_batch(n_nodes, seed, mult=(1, 2, 3, 9, 40, 700, 1300)):
    """A pod batch of repeated rows: shapes of the config-2 distribution, each repeated `mult` times in a
    shuffled queue (a row of 1,300 pods spans several k_eval3_dup work items), plus distinct singles."""
    rng = np.random.default_rng(seed)
    base = synth.make_cluster(n_nodes, 400, seed=seed)
    picks = [rng.integers(0, 400) for _ in mult for _ in range(3)]
    reps = np.repeat(picks, [m for m in mult for _ in range(3)])
    order = np.concatenate([reps, np.arange(400)])   # the 400 originals: mostly singles or small groups
    rng.shuffle(order)
    pods = base.pods.copy()
    view = base.with_nodes(base.nodes, pods)
    return view, order


@pytest.mark.parametrize("profile", ["shipped", "most_w", "prod_usage"])
def test_matrix_parity_duplicate_rows(profile):
    """k_eval3_dup: pods whose class rows repeat are evaluated once per distinct row and written to every pod
    of the row (multiplicities 2 to 1,300, work items split inside a row, singles on the plain path); planes,
    top-1 and a top-1-only pass against the oracle on a ragged cluster with slow nodes."""
    cfg = {"shipped": shipped_profile, "prod_usage": lambda: shipped_profile(score_according_prod_usage=True),
           "most_w": lambda: make_config(fit_strategy="MostAllocated", fit_resources={"cpu": 2, "memory": 1})}[profile]()
    cl, order = _dup_batch(2_500, 41)
    big = np.arange(5, 2_500, 83)
    cl.nodes["allocatable"]["v"][big, 1] = (1 << 43) + 99
    cl = cl.with_nodes(cl.nodes)
    _check_matrix(cfg, cl, order, cl.now_ns)
    with _engine_for(cfg, cl, order) as eng:
        full = eng.eval(cl.now_ns)
        keys = eng.eval(cl.now_ns, mask=False, scores=False)
    np.testing.assert_array_equal(keys["top1"], full["top1"])


@pytest.mark.parametrize("n_nodes", [1, 63, 64, 511, 513, 1500])
def test_matrix_parity_ragged_node_counts(n_nodes):
    cl = synth.make_cluster(n_nodes, 70, seed=n_nodes)
    _check_matrix(shipped_profile(), cl, np.arange(70), cl.now_ns)


def test_matrix_slow_path_huge_nodes():
    """Nodes beyond the fp64 fast-path bounds (cap >= 2^41 B) take the exact int64 path."""
    cl = synth.make_cluster(700, 40, seed=5)
    big = np.arange(0, 700, 7)
    cl.nodes["allocatable"]["v"][big, 1] = (1 << 43) + 12345
    cl.nodes["requested"]["v"][big, 1] = (1 << 42) + 777
    cl.nodes["nonzero_requested"][big, 1] = (1 << 42) + 777
    cl = cl.with_nodes(cl.nodes)
    _check_matrix(shipped_profile(), cl, np.arange(40), cl.now_ns)


def test_matrix_daemonset_and_prod_score_variant():
    cl = synth.make_cluster(1_000, 64, seed=9)
    cl.pods["is_daemonset"][::5] = 1
    cl = cl.with_nodes(cl.nodes)
    cfg = shipped_profile(score_according_prod_usage=True, prod_usage_thresholds={"cpu": 40})
    _check_matrix(cfg, cl, np.arange(64), cl.now_ns)


def test_empty_pod_batch():
    cl = synth.make_cluster(600, 1, seed=3)
    cfg = shipped_profile()
    with _engine_for(cfg, cl, []) as eng:
        res = eng.eval(cl.now_ns)
        assert res["mask"].shape[0] == 0
        nodes, scores = eng.place(cl.now_ns)
        assert len(nodes) == 0


@pytest.mark.parametrize("chunk", [1, 7, 64])
def test_placement_matches_sequential_cycle(chunk):
    cl = synth.make_cluster(3_000, 400, seed=21)
    cfg = shipped_profile(place_chunk=chunk)
    idx = np.arange(400)
    with _engine_for(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_nodes, ref_scores = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    # snapshot rows after the commits equal host-side Reserve deltas
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    np.testing.assert_array_equal(after, rows)


@pytest.mark.parametrize("chunk", [15, 16, 17])
def test_placement_slow_nodes_and_list_depth(chunk):
    """Placement with nodes outside the fp64 bounds from the start (cap ≥ 2^41 B) and nodes whose score
    base crosses 2^50 on their first commit (the resolve lists them as slow), at chunk sizes around the
    top-k list depth (KG_PARTIAL_SLOTS = 16: a 17th pod can find every listed node of a tile touched)."""
    cl = synth.make_cluster(2_500, 300, seed=24)
    big = np.arange(0, 2_500, 11)
    cl.nodes["allocatable"]["v"][big, 1] = (1 << 43) + 12345
    cl.nodes["requested"]["v"][big, 1] = (1 << 42) + 777
    cl.nodes["nonzero_requested"][big, 1] = (1 << 42) + 777
    edge = np.arange(5, 2_500, 13)
    cl.nodes["nonzero_requested"][edge, 1] = (1 << 50) - (64 << 20)
    cl = cl.with_nodes(cl.nodes)
    # MostAllocated: a huge score base clamps to 100, so the edge nodes attract pods and cross the bound
    cfg = shipped_profile(place_chunk=chunk, fit_strategy="MostAllocated")
    idx = np.arange(300)
    with _engine_for(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_nodes, ref_scores = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    assert np.isin(nodes, big).any() and np.isin(nodes, edge).any()
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    np.testing.assert_array_equal(after, rows)


def test_placement_tight_cluster_with_unschedulable_pods():
    """Few small nodes: pods run out of room, later pods become unschedulable (−1)."""
    cl = synth.make_cluster(10, 1200, seed=33, no_metric_frac=0.3)
    cfg = shipped_profile(place_chunk=32)
    idx = np.arange(1200)
    with _engine_for(cfg, cl, idx) as eng:
        nodes, scores = eng.place(cl.now_ns)
    ref_nodes, ref_scores = oracle.schedule(cfg, cl, idx, cl.now_ns)
    assert (ref_nodes == -1).any()
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)


def test_snapshot_upsert_remove_and_commit():
    cl = synth.make_cluster(2_000, 50, seed=8)
    cfg = shipped_profile()
    idx = np.arange(50)
    rows = engine.build_node_rows(cfg, cl)
    with _engine_for(cfg, cl, idx) as eng:
        eng.remove(17)
        eng.commit(3, 99)
        res = eng.eval(cl.now_ns)
        got = eng.download()
    prow = engine.build_pod_rows(cfg, cl, idx)
    engine.row_commit(cfg, rows[99:100], prow[3:4])
    np.testing.assert_array_equal(got[99], rows[99])
    assert got[17]["flags"] == 0
    mask = engine.unpack_mask(res["mask"], 2000)
    assert not mask[:, 17].any()


def test_snapshot_generation_counts_mutations():
    """kg_snapshot_generation: reset, upsert / remove, commit and each placement resolve
    advance it; evaluations do not."""
    cl = synth.make_cluster(1_500, 16, seed=9)
    cfg = shipped_profile(place_chunk=8)
    idx = np.arange(16)
    with engine.Engine(cfg) as eng:
        assert eng.generation() == 0
        eng.load_snapshot(engine.build_node_rows(cfg, cl))       # reset + upsert
        g0 = eng.generation()
        assert g0 == 2
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        eng.eval(cl.now_ns)
        assert eng.generation() == g0
        eng.remove(5)
        eng.commit(0, 7)
        assert eng.generation() == g0 + 2
        eng.place(cl.now_ns)                                      # 16 pods in 8-pod chunks: 2 resolves
        assert eng.generation() == g0 + 4


def test_debug_scores_dump_from_engine(monkeypatch, caplog):
    """KOORD_GPU_DEBUG_TOPN (frameworkext/debug.go --debug-scores): Engine.eval logs one top-N table per
    pod; its first row is the pod's top-1 and its totals are the oracle's weighted sums."""
    import logging
    monkeypatch.setenv("KOORD_GPU_DEBUG_TOPN", "5")
    cl = synth.make_cluster(600, 12, seed=5)
    cfg = shipped_profile()
    with caplog.at_level(logging.INFO, logger="koordinator_amd.debug"):
        with _engine_for(cfg, cl, np.arange(12)) as eng:
            res = eng.eval(cl.now_ns)
    tables = [r.getMessage() for r in caplog.records if r.name == "koordinator_amd.debug"]
    assert len(tables) == 12
    m_ref, fit_ref, la_ref = oracle.eval_matrix(cfg, cl, np.arange(12), cl.now_ns)
    node, tot = engine.decode_top1(res["top1"])
    for p, t in enumerate(tables):
        rows = [ln for ln in t.splitlines() if ln.startswith("| 0 |") or ln.startswith("| 1 |")]
        cells = rows[0].split(" | ")
        assert cells[2] == f"node-{node[p]}" and int(cells[3]) == tot[p]
        total = np.where(m_ref[p], fit_ref[p].astype(int) * int(cfg["weight_fit"]) + la_ref[p].astype(int) * int(cfg["weight_loadaware"]), -1)
        assert sorted(total[m_ref[p]], reverse=True)[:2] == [int(r.split(" | ")[3]) for r in rows]
