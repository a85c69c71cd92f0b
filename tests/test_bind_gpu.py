"""NodeNUMAResource cpuset binding through kg_eval on the GPU (matrix mode; nodes with and without a NUMA
topology policy) against the oracle's literal Allocate (CPU accumulator pinned by cpu_accumulator_test.go),
with NodeResourcesFit and LoadAwareScheduling in the profile; and placement with the cpuset Reserve (kg_place /
kg_commit; the host takes the CPUs) against the oracle's literal cycle.  The paths the engine does not take (the
sharded chunk API with cpusets, cpusets with Reservation) are refused, not answered."""
import numpy as np
import pytest

from bind_cases import make_bind_cluster
from koordinator_amd import _native as nat
from koordinator_amd import engine
from koordinator_amd.config import shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu


def _cfg(**kw):
    cfg = shipped_profile(**kw)
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    return cfg


@pytest.mark.parametrize("seed,n_nodes,n_pods,numa_frac", [(1, 300, 96, 0.35), (2, 1100, 70, 0.35), (3, 64, 200, 0.35),
                                                            (5, 700, 90, 1.0)])
def test_bind_matrix_matches_oracle(seed, n_nodes, n_pods, numa_frac):
    cl, view, idx = make_bind_cluster(n_nodes, n_pods, seed, numa_frac=numa_frac)
    cfg = _cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_pods(engine.build_pod_rows(cfg, view, idx))
        res = eng.eval(cl.now_ns)
    m, f, l, n = oracle.eval_matrix3(cfg, view, np.asarray(idx), cl.now_ns)
    N = len(cl.nodes)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], f)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], l)
    np.testing.assert_array_equal(res["numa_scores"][:, :N], n)
    tot = np.where(m, f.astype(np.int64) + l.astype(np.int64) + int(cfg["weight_numa"]) * n.astype(np.int64), -1)
    node, best = engine.decode_top1(res["top1"])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    assert 0.05 < m.mean() < 0.95


@pytest.mark.parametrize("seed,n_nodes,n_pods,numa_frac,chunk", [(21, 300, 200, 0.35, 16), (22, 1100, 150, 1.0, 16),
                                                                  (23, 200, 300, 0.0, 4), (24, 700, 250, 0.5, 64)])
def test_bind_placement_matches_oracle(seed, n_nodes, n_pods, numa_frac, chunk):
    """kg_place with cpuset Reserve (the host takes the CPUs between device chunks) against the oracle's literal
    cycle: placements, scores, every node's CPUs after the last Reserve, and the rows (host replay through the
    engine's per-pair code)."""
    from reserve_cycle import cpu_tables, host_cycle
    cl, view, idx = make_bind_cluster(n_nodes, n_pods, seed, numa_frac=numa_frac)
    cfg = _cfg()
    cfg["place_chunk"] = chunk
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_cpus(view)
        eng.set_pods(engine.build_pod_rows(cfg, view, idx))
        nodes, scores = eng.place(cl.now_ns)
        rows = eng.download()
        tabs = cpu_tables(view)
        got_cpus = view.cpu_arr.copy()
        for j, (first, n, _, _) in tabs.items():
            got_cpus[first:first + n] = eng.download_cpus(j, n)
    ref_nodes, ref_scores, ref_cpus = oracle.schedule_cpus(cfg, view, np.asarray(idx), cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(got_cpus, ref_cpus)
    _, _, ref_rows, _ = host_cycle(cfg, view, idx, cl.now_ns)
    assert rows.tobytes() == ref_rows.tobytes()
    assert int((got_cpus["refcount"] != view.cpu_arr["refcount"]).sum()) > 0


def test_bind_reserve_failure_gpu():
    """A Reserve that fails after its Filter passed: kg_place leaves the pod unplaced and unchanged state;
    kg_commit reports it (False) and changes nothing."""
    from bind_cases import make_reserve_fail_cluster
    cl, view, idx = make_reserve_fail_cluster()
    cfg = _cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_cpus(view)
        eng.set_pods(engine.build_pod_rows(cfg, view, idx))
        nodes, scores = eng.place(cl.now_ns)
        assert nodes.tolist() == [-1, 0, 0]
        assert np.flatnonzero(eng.download_cpus(0, 8)["refcount"]).tolist() == [2, 3, 4, 5, 6, 7]
        ref_nodes, ref_scores, _ = oracle.schedule_cpus(cfg, view, np.asarray(idx), cl.now_ns)
        np.testing.assert_array_equal(scores, ref_scores)
        # kg_commit on a fresh snapshot: the 8-CPU pod fails, the 2-CPU pod takes cores 1
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_cpus(view)
        before = eng.download()
        assert eng.commit(0, 0) is False
        assert eng.download().tobytes() == before.tobytes()
        assert eng.commit(1, 0) is True
        assert np.flatnonzero(eng.download_cpus(0, 8)["refcount"]).tolist() == [2, 3]


def test_bind_chunk_api_and_reservation_are_refused():
    """The sharded chunk API has no host Reserve step; cpusets with Reservation are not on the engine path."""
    cl, view, idx = make_bind_cluster(128, 8, 4)
    cfg = _cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_pods(engine.build_pod_rows(cfg, view, idx))
        with pytest.raises(engine.EngineError, match="kg_cpus_set"):
            eng.place(cl.now_ns)   # the CPU tables were never set
        eng.set_cpus(view)
        with pytest.raises(engine.EngineError, match="chunk API"):
            eng.chunk_eval(cl.now_ns, 0, 4, 0)
        eng.eval(cl.now_ns)   # matrix mode still answers
    cfg2 = _cfg()
    cfg2["enabled_plugins"] |= nat.PLUGIN_RESERVATION
    with engine.Engine(cfg2) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg2, view))
        eng.set_cpus(view)
        eng.set_pods(engine.build_pod_rows(cfg2, view, idx))
        with pytest.raises(engine.EngineError, match="Reservation"):
            eng.place(cl.now_ns)


def test_numa_plugin_filter_kat_gpu():
    """TestPlugin_Filter (plugin_test.go:552-899) through kg_eval, the SingleNUMANode cpuset cases included."""
    from test_numa_plugin_filter_kat import DOC, _cluster
    for case in DOC["cases"]:
        cfg, view, pi = _cluster(case)
        with engine.Engine(cfg) as eng:
            eng.load_snapshot(engine.build_node_rows(cfg, view))
            eng.set_pods(engine.build_pod_rows(cfg, view, [pi]))
            res = eng.eval(0)
        assert bool(engine.unpack_mask(res["mask"], 1)[0, 0]) == case["want"], case["name"]
