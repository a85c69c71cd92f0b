"""Pin the CPU oracle (and the host row builders) to the reference's own known-answer tests."""
import numpy as np
import pytest

from kat import case_cluster, load, pod_from
from koordinator_amd import engine
from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Node
from oracle import oracle

DOC = load("loadaware_kat.json")


@pytest.mark.parametrize("case", DOC["score_cases"], ids=lambda c: c["name"])
def test_oracle_loadaware_score_kat(case):
    cfg, view, pi, cl = case_cluster(DOC, case, "pod")
    assert oracle.la_score(cfg, view, pi, 0, cl.now_ns) == case["want"]


@pytest.mark.parametrize("case", DOC["filter_cases"], ids=lambda c: c["name"])
def test_oracle_loadaware_filter_kat(case):
    cfg, view, pi, cl = case_cluster(DOC, case, "test_pod")
    assert oracle.la_filter(cfg, view, pi, 0, cl.now_ns) == case["want"]


@pytest.mark.parametrize("case", DOC["estimate_pod_cases"], ids=lambda c: c["name"])
def test_pod_row_estimate_kat(case):
    """EstimatePod (default_estimator.go:57-108) through the product's host row builder."""
    cfg = make_config(estimated_scaling_factors=case.get("scaling"))
    cl = Cluster()
    cl.add_node(Node("n", allocatable={"cpu": "1"}))
    pod = pod_from(case["pod"])
    view = cl.view(extra_pods=[pod])
    row = engine.build_pod_rows(cfg, view, [view.pod_index(pod)])[0]
    assert int(row["la_estimate"][0]) == case["want"]["cpu"]
    assert int(row["la_estimate"][1]) == case["want"]["memory"]


@pytest.mark.parametrize("case", DOC["estimate_node_cases"], ids=lambda c: c["name"])
def test_node_row_estimate_kat(case):
    """EstimateNode (default_estimator.go:110-129) through the product's host row builder."""
    cfg = make_config()
    cl = Cluster()
    cl.add_node(Node("n", allocatable=case["allocatable"], annotations_raw_allocatable=case.get("raw_allocatable")))
    view = cl.view()
    row = engine.build_node_rows(cfg, view)[0]
    assert int(row["la_alloc"][0]) == case["want"]["cpu"]
    assert int(row["la_alloc"][1]) == case["want"]["memory"]
