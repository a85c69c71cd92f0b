"""NodeNUMAResource cpuset binding through kg_eval on the GPU (matrix mode; nodes with and without a NUMA
topology policy) against the oracle's literal Allocate (CPU accumulator pinned by cpu_accumulator_test.go),
with NodeResourcesFit and LoadAwareScheduling in the profile; the path the engine does not take (the Reserve
of a cpuset) is refused, not answered."""
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


def test_bind_placement_is_refused():
    cl, view, idx = make_bind_cluster(128, 8, 4)
    cfg = _cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_pods(engine.build_pod_rows(cfg, view, idx))
        with pytest.raises(engine.EngineError, match="cpuset"):
            eng.place(cl.now_ns)
        with pytest.raises(engine.EngineError, match="cpuset"):
            eng.commit(0, 0)
        eng.eval(cl.now_ns)   # matrix mode still answers


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
