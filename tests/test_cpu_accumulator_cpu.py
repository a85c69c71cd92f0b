"""NodeNUMAResource cpuset take (oracle/cpu_accumulator.c) pinned by the reference's own tests
(tests/golden/cpu_accumulator_kat.json, transcribed from cpu_accumulator_test.go by
tests/golden/make_cpu_accumulator_kat.py)."""
import numpy as np
import pytest

from kat import load
from oracle import oracle

DOC = load("cpu_accumulator_kat.json")


@pytest.mark.parametrize("case", DOC["table"], ids=lambda c: f"{c['test']}/{c['name']}")
def test_take_cpus_kat(case):
    topo = oracle.test_topology(*case["topology"])
    n = len(topo[0])
    allocated = set(case["allocated"])
    excl = np.zeros(n, np.int8)
    if case["allocated_exclusive"]:
        for c in allocated:
            excl[c] = oracle.EXCLUSIVE[case["allocated_exclusive"]]
    got = oracle.take_cpus(topo, case["max_ref"], [c for c in range(n) if c not in allocated], case["need"],
                           case["bind"], case["excl"], case["strategy"], alloc_excl=excl)
    if case["want_error"]:
        assert got is None
    else:
        assert got == case["want"]


@pytest.mark.parametrize("seq", DOC["sequential"], ids=lambda s: s["name"])
def test_take_cpus_with_ref_counts(seq):
    """Successive pods on one NodeAllocation with maxRefCount 2: getAvailableCPUs → takeCPUs → addCPUs."""
    topo = oracle.test_topology(*seq["topology"])
    n = len(topo[0])
    ref = np.zeros(n, np.int32)
    excl = np.zeros(n, np.int8)
    for step in seq["steps"]:
        available = [c for c in range(n) if ref[c] < seq["max_ref"]]
        got = oracle.take_cpus(topo, seq["max_ref"], available, step["need"], step["bind"], "None",
                               "MostAllocated", alloc_ref=ref, alloc_excl=excl)
        assert got == step["want"]
        for c in got:                       # addCPUs(…, CPUExclusivePolicyPCPULevel)
            ref[c] += 1
            excl[c] = oracle.EXCLUSIVE["PCPULevel"]
    if "want_available_after" in seq:
        assert [c for c in range(n) if ref[c] < seq["max_ref"]] == seq["want_available_after"]


@pytest.mark.parametrize("i", range(len(DOC["preferred"]["cases"])))
def test_take_preferred_cpus(i):
    topo = oracle.test_topology(*DOC["preferred"]["topology"])
    n = len(topo[0])
    c = DOC["preferred"]["cases"][i]
    available = list(range(n)) if c["available"] == "all" else [x for x in range(n) if x not in (0, 2)]
    got = oracle.take_cpus(topo, 1, available, c["need"], "SpreadByPCPUs", preferred=c["preferred"])
    assert got == c["want"]


def test_take_more_than_available_fails():
    topo = oracle.test_topology(1, 1, 4, 2)
    assert oracle.take_cpus(topo, 1, range(4), 5, "SpreadByPCPUs") is None
    assert oracle.take_cpus(topo, 1, range(8), 0, "FullPCPUs") == []
