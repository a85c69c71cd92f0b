"""ElasticQuota PreFilter known answers (TestPlugin_PreFilter, TestPlugin_Prefilter_QuotaNonPreempt,
TestPlugin_PreFilter_CheckParent) through the oracle's cycle (mask of a one-node cluster) and, on the GPU, through kg_eval."""
import numpy as np
import pytest

from koordinator_amd import engine, synth
from oracle import oracle
from quota_cases import doc, quota_config, quota_view

DOC = doc()


@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_quota_prefilter_kat_oracle(case):
    view, cfg = quota_view(case), quota_config(case)
    m, *_ = oracle.eval_matrix5(cfg, view, np.arange(1), view.now_ns)
    assert bool(m[0, 0]) == case["want"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_quota_prefilter_kat_gpu(case):
    view, cfg = quota_view(case), quota_config(case)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_quotas(view.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, view, [0]))
        res = eng.eval(view.now_ns)
        nodes, _ = eng.place(view.now_ns)
    assert bool(engine.unpack_mask(res["mask"], 1)[0, 0]) == case["want"]
    assert (nodes[0] == 0) == case["want"]


from quota_cases import used_tree_doc, used_tree_view, used_tree_want  # noqa: E402

TREE = used_tree_doc()


def _tree_cfg():
    from koordinator_amd.config import make_config
    return make_config(plugins=("NodeResourcesFit", "ElasticQuota"), eq_check_parent_quota=1)


@pytest.mark.parametrize("case", TREE["cases"], ids=lambda c: c["name"])
def test_quota_used_tree_kat_oracle(case):
    """Reserve adds a pod's request to its group and every ancestor (used, and nonPreemptibleUsed for a
    non-preemptible pod): group_quota_manager_test.go's used-delta cases through the oracle's cycle."""
    view, names = used_tree_view(case)
    nodes, _, _, q = oracle.schedule2(_tree_cfg(), view, np.arange(len(case["pods"])), view.now_ns)
    assert (nodes == 0).all()
    for g, (used, npu) in enumerate(used_tree_want(case, names)):
        np.testing.assert_array_equal(q["used"]["v"][g], used, err_msg=names[g])
        np.testing.assert_array_equal(q["non_preemptible_used"]["v"][g], npu, err_msg=names[g])


@pytest.mark.gpu
@pytest.mark.parametrize("case", TREE["cases"], ids=lambda c: c["name"])
def test_quota_used_tree_kat_gpu(case):
    view, names = used_tree_view(case)
    cfg = _tree_cfg()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, view))
        eng.set_quotas(view.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, view, np.arange(len(case["pods"]))))
        nodes, _ = eng.place(view.now_ns)
        q = eng.download_quotas()
    assert (nodes == 0).all()
    for g, (used, npu) in enumerate(used_tree_want(case, names)):
        np.testing.assert_array_equal(q["used"]["v"][g], used, err_msg=names[g])
        np.testing.assert_array_equal(q["non_preemptible_used"]["v"][g], npu, err_msg=names[g])


def test_oracle_rejects_invalid_quota_tree():
    """The oracle validates parent chains like kg_quota_set (no out-of-range, self or cyclic parent)
    instead of walking out of the array."""
    case = TREE["cases"][0]
    for parents in ([1, 2, 0], [-1, 7, 1], [0, 0, 1]):
        view, _ = used_tree_view(case)
        q = view.quota_arr.copy()
        q["parent"] = parents
        bad = synth.SynthView(view.pods, view.containers, view.nodes, view.now_ns, quotas=q)
        with pytest.raises(RuntimeError, match="kgo_schedule2 failed"):
            oracle.schedule2(_tree_cfg(), bad, np.arange(len(case["pods"])), bad.now_ns)
