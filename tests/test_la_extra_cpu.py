"""LoadAwareScheduling resourceWeights beyond cpu / memory (load_aware.go:378-397 loadAwareSchedulingScorer
over every weighted resource; default_estimator.go:57-108 EstimatePod per weighted resource, with the
priority-class name translation of apis/extension/resource.go:53-58) on the host: the engine's per-pair
exact code (kg_row_eval → kg_pair_exact) and Reserve (kg_row_commit) against the oracle restatement.

The reference's own LoadAware tests use cpu / memory weights only, so beyond those two resources this
is parity against the oracle's restatement (parity unpinned upstream)."""
import numpy as np
import pytest

from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle

WEIGHTS = {
    "eph+gpu": {"cpu": 1, "memory": 1, "ephemeral-storage": 1, "example.com/gpu": 2},
    "batch": {"cpu": 2, "memory": 1, "kubernetes.io/batch-cpu": 1, "kubernetes.io/batch-memory": 3},
    "eph only": {"ephemeral-storage": 1},
}


def _config(weights, shipped=False, **kw):
    kw = dict(resource_weights=weights, estimated_scaling_factors={"ephemeral-storage": 60, "example.com/gpu": 100},
              **kw)
    return shipped_profile(**kw) if shipped else make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling"), **kw)


def _pairs(cfg, cl, P, N):
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    out = np.zeros((3, P, N), np.int64)
    for i in range(P):
        for j in range(N):
            out[:, i, j] = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)[:3]
    return out


@pytest.mark.parametrize("name", sorted(WEIGHTS))
@pytest.mark.parametrize("shipped", [False, True], ids=["default", "shipped"])
def test_row_eval_la_extra_matches_oracle(name, shipped):
    P, N = 40, 150
    cl = synth.make_la_extra_cluster(N, P, seed=31)
    cfg = _config(WEIGHTS[name], shipped=shipped, score_according_prod_usage=shipped)
    got = _pairs(cfg, cl, P, N)
    m, f, l = oracle.eval_matrix(cfg, cl, np.arange(P), cl.now_ns)
    np.testing.assert_array_equal(got[0].astype(bool), m)
    np.testing.assert_array_equal(got[1], f)
    np.testing.assert_array_equal(got[2], l)
    # the extra resources move the LoadAware score: it differs from the cpu / memory-only one somewhere
    base = oracle.eval_matrix(_config({"cpu": 1, "memory": 1}, shipped=shipped), cl, np.arange(P), cl.now_ns)[2]
    assert (base != l).any()


def test_pod_rows_carry_extra_estimates():
    cl = synth.make_la_extra_cluster(50, 60, seed=32)
    cfg = _config(WEIGHTS["eph+gpu"])
    pods = engine.build_pod_rows(cfg, cl, np.arange(60))
    nodes = engine.build_node_rows(cfg, cl)
    assert (pods["la_estimate_x"][:, 0] > 0).any()        # ephemeral-storage estimate
    assert (pods["la_estimate_x"][:, 5] > 0).any()        # example.com/gpu estimate
    assert (nodes["la_alloc_x"][:, 0] > 0).any() and (nodes["la_used_x"][:, 0, 0] > 0).any()
    plain = engine.build_pod_rows(_config({"cpu": 1, "memory": 1}), cl, np.arange(60))
    assert not plain["la_estimate_x"].any()               # only weighted resources are estimated


@pytest.mark.parametrize("seed", [33, 34])
def test_row_commit_la_extra_matches_sequential_oracle(seed):
    """Sequential cycle over host rows (kg_row_eval + kg_row_commit) == kgo_schedule with the extra
    resources' estimates added to the node terms by each Reserve."""
    P, N = 60, 30
    cl = synth.make_la_extra_cluster(N, P, seed=seed)
    cfg = _config(WEIGHTS["eph+gpu"])
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    got_n, got_s = [], []
    for i in range(P):
        best, bn = -1, -1
        for j in range(N):
            ok, fit, la, _ = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)
            tot = int(cfg["weight_fit"]) * fit + int(cfg["weight_loadaware"]) * la
            if ok and tot > best:
                best, bn = tot, j
        if bn >= 0:
            engine.row_commit(cfg, nodes[bn:bn + 1], pods[i:i + 1])
        got_n.append(bn)
        got_s.append(best)
    ref_n, ref_s = oracle.schedule(cfg, cl, np.arange(P), cl.now_ns)
    np.testing.assert_array_equal(np.array(got_n), ref_n)
    np.testing.assert_array_equal(np.array(got_s), ref_s)
    assert (ref_n >= 0).sum() > P // 2
