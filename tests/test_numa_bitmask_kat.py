"""Topology-manager known answers (tests/golden/numa_bitmask_filter_kat.json): filterSingleNumaHints
(TestPolicySingleNumaNodeFilterHints), IsNarrowerThan through the merge (TestIsNarrowerThan) and the
IterateBitMasks enumeration through generateResourceHints (TestIterateBitMasks), on the oracle."""
import itertools

import pytest

from kat import load
from koordinator_amd import _native as nat
from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Container, Node, Pod
from oracle import oracle

DOC = load("numa_bitmask_filter_kat.json")


def _bits(b):
    return None if b is None else sum(1 << x for x in b)


@pytest.mark.parametrize("case", DOC["filter_single"], ids=lambda c: c["name"])
def test_filter_single_numa_hints_kat(case):
    lists = [[(_bits(m), p) for m, p in l] for l in case["all"]]
    want = [[(_bits(m), p) for m, p in l] for l in case["want"]]
    assert oracle.filter_single_numa_hints(lists) == want


@pytest.mark.parametrize("case", DOC["narrower"], ids=lambda c: c["name"])
def test_is_narrower_than_kat(case):
    first, second = case["first"], case["second"]
    admit, bits, pref = oracle.numa_merge(nat.NUMA_BEST_EFFORT, [0, 1], [[(second, True), (first, True)]])
    assert admit and pref
    assert (bits == first) == case["want"]


@pytest.mark.parametrize("case", DOC["iterate"], ids=lambda c: c["name"])
def test_iterate_bit_masks_kat(case):
    n = case["bits"]
    node = Node("n", allocatable={"cpu": f"{8 * n}", "memory": f"{8 * n}Gi"}, numa_policy="BestEffort")
    node.numa_zones = [{"cpu": "8", "memory": "8Gi"} for _ in range(n)]
    node.numa_zone_ids = list(range(n))
    cl = Cluster()
    cl.add_node(node)
    pod = Pod(name="p", containers=[Container(requests={"cpu": "1"})])
    view = cl.view(extra_pods=[pod])
    lists = oracle.numa_hint_lists(make_config(plugins=("NodeNUMAResource",)), view, view.pod_index(pod), 0)
    masks = [m for m, _ in lists[nat.RES_CPU]]
    assert len(masks) == (1 << n) - 1
    assert masks == [sum(1 << b for b in c) for k in range(1, n + 1) for c in itertools.combinations(range(n), k)]
