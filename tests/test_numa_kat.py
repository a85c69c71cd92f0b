"""Pin the NodeNUMAResource restatement (oracle) to the reference's own known-answer tests.

* topology-manager merge: every case of frameworkext/topologymanager/policy_test.go (common, best-effort /
  restricted and single-numa-node groups) through oracle.numa_merge;
* NodeNUMAResource Filter + Score: TestNUMANodeScore (nodenumaresource/scoring_test.go:47-330).
"""
import pytest

from kat import load
from numa_kat import merge_lists, numa_score_cluster
from koordinator_amd import _native as nat
from oracle import oracle

MERGE = load("numa_merge_kat.json")
SCORE = load("numa_score_kat.json")
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
