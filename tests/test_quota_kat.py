"""ElasticQuota PreFilter known answers (TestPlugin_PreFilter, TestPlugin_Prefilter_QuotaNonPreempt,
TestPlugin_PreFilter_CheckParent) through the oracle's cycle (mask of a one-node cluster) and, on the GPU, through kg_eval."""
import numpy as np
import pytest

from koordinator_amd import engine
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
