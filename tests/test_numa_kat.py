"""Pin the NodeNUMAResource restatement (oracle) to the reference's own known-answer tests.

* topology-manager merge: every case of frameworkext/topologymanager/policy_test.go (common, best-effort /
  restricted and single-numa-node groups) through oracle.numa_merge;
* NodeNUMAResource Filter + Score: TestNUMANodeScore (nodenumaresource/scoring_test.go:47-330);
* amplified CPUs with cpuset pods on the node: TestScoreWithAmplifiedCPUs (scoring_test.go:556-835) and
  TestFilterWithAmplifiedCPUs (plugin_test.go:901-1012); the cases whose scheduled pod binds a cpuset
  are outside the engine path and checked to be rejected (test_numa_rows_cpu.py).
"""
import pytest

from kat import load
from numa_kat import amplified_filter_cluster, amplified_score_cluster, merge_lists, numa_score_cluster
from koordinator_amd import _native as nat
from oracle import oracle

MERGE = load("numa_merge_kat.json")
SCORE = load("numa_score_kat.json")
AMP = load("numa_amplified_kat.json")
POLICY = {"BestEffort": nat.NUMA_BEST_EFFORT, "Restricted": nat.NUMA_RESTRICTED,
          "SingleNUMANode": nat.NUMA_SINGLE_NUMA_NODE}


@pytest.mark.parametrize("case", [(c, p) for c in MERGE["cases"] for p in c["policies"]],
                         ids=lambda cp: f"{cp[1]}:{cp[0]['name']}")
def test_oracle_numa_merge_kat(case):
    c, policy = case
    admit, bits, pref = oracle.numa_merge(POLICY[policy], MERGE["numa_nodes"], merge_lists(c["providers"]))
    assert bits == c["want"]["mask"]
    assert pref == c["want"]["preferred"]
    assert admit == (True if policy == "BestEffort" else pref)


@pytest.mark.parametrize("case", SCORE["cases"], ids=lambda c: c["name"])
def test_oracle_numa_score_kat(case):
    cfg, view, pi, cl = numa_score_cluster(case)
    got = []
    for j in range(len(case["nodes"])):
        ok, score = oracle.numa_eval(cfg, view, pi, j)
        assert ok
        got.append(score)
    assert got == case["want"]


@pytest.mark.parametrize("case", AMP["score_cases"], ids=lambda c: c["name"])
def test_oracle_amplified_score_kat(case):
    cfg, view, pi, cl = amplified_score_cluster(case)
    got = []
    for j in range(len(case["nodes"])):
        ok, score = oracle.numa_eval(cfg, view, pi, j)
        assert ok
        got.append(score)
    assert got == case["want"]


@pytest.mark.parametrize("case", AMP["filter_cases"], ids=lambda c: c["name"])
def test_oracle_amplified_filter_kat(case):
    cfg, view, pi, cl = amplified_filter_cluster(case)
    ok, _ = oracle.numa_eval(cfg, view, pi, 0)
    assert ok == case["want"]
