"""ElasticQuota PreFilter known answers (TestPlugin_PreFilter, TestPlugin_Prefilter_QuotaNonPreempt)
through the oracle's cycle (mask of a one-node cluster) and, on the GPU, through kg_eval."""
import numpy as np
import pytest

from koordinator_amd import engine
from koordinator_amd.config import make_config
from oracle import oracle
from quota_cases import doc, quota_view

DOC = doc()
CFG = make_config(plugins=("NodeResourcesFit", "ElasticQuota"))


@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_quota_prefilter_kat_oracle(case):
    view = quota_view(case)
    m, *_ = oracle.eval_matrix5(CFG, view, np.arange(1), view.now_ns)
    assert bool(m[0, 0]) == case["want"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_quota_prefilter_kat_gpu(case):
    view = quota_view(case)
    with engine.Engine(CFG) as eng:
        eng.load_snapshot(engine.build_node_rows(CFG, view))
        eng.set_quotas(view.quota_arr)
        eng.set_pods(engine.build_pod_rows(CFG, view, [0]))
        res = eng.eval(view.now_ns)
        nodes, _ = eng.place(view.now_ns)
    assert bool(engine.unpack_mask(res["mask"], 1)[0, 0]) == case["want"]
    assert (nodes[0] == 0) == case["want"]
