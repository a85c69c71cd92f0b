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


# ---- the product's accumulator (kg_cpuset.cpp through the C-ABI's kg_cpuset_take), pinned by the same cases ----
# (host code: runs on the CPU; the oracle's C copy above is the checker for everything else, this pins the
# engine's own restatement directly against the reference's expectations)

from koordinator_amd import _native as nat  # noqa: E402

ABI_BIND = {"": nat.CPU_BIND_UNSET, "FullPCPUs": nat.CPU_BIND_FULL_PCPUS, "SpreadByPCPUs": nat.CPU_BIND_SPREAD_BY_PCPUS}
ABI_EXCL = {"": nat.CPU_EXCL_UNSET, "None": nat.CPU_EXCL_NONE, "PCPULevel": nat.CPU_EXCL_PCPU_LEVEL,
            "NUMANodeLevel": nat.CPU_EXCL_NUMA_NODE_LEVEL}
ABI_STRATEGY = {"LeastAllocated": nat.STRATEGY_LEAST_ALLOCATED, "MostAllocated": nat.STRATEGY_MOST_ALLOCATED}


def _product_take(topo, max_ref, available, need, bind, excl="None", strategy="MostAllocated", ref=None, alloc_excl=None):
    s, n_, c = topo
    n = len(s)
    cpus = np.zeros(n, dtype=nat.CPU_INFO)
    cpus["socket"], cpus["node"], cpus["core"] = s, n_, c
    if ref is not None:
        cpus["refcount"] = ref
    if alloc_excl is not None:
        cpus["exclusive"] = [ABI_EXCL[x] for x in alloc_excl]
    av = np.zeros(n, np.uint8)
    av[list(available)] = 1
    out = np.zeros(n, np.uint8)
    st = nat.lib().kg_cpuset_take(nat.ptr(cpus), n, max_ref, nat.ptr(av), need, ABI_BIND[bind], ABI_EXCL[excl],
                                  ABI_STRATEGY[strategy], nat.ptr(out))
    assert st in (0, 1), st   # KG_OK / KG_NOT_FOUND
    return None if st == 1 else [int(i) for i in np.flatnonzero(out)]


@pytest.mark.parametrize("case", DOC["table"], ids=lambda c: f"{c['test']}/{c['name']}")
def test_product_take_cpus_kat(case):
    topo = oracle.test_topology(*case["topology"])
    n = len(topo[0])
    allocated = set(case["allocated"])
    ref = np.zeros(n, np.int32)
    excl = ["" for _ in range(n)]
    for c in allocated:
        ref[c] = 1   # allocated CPUs of these cases are unavailable (maxRefCount 1) and carry their policy
        excl[c] = case["allocated_exclusive"] or ""
    got = _product_take(topo, case["max_ref"], [c for c in range(n) if c not in allocated], case["need"], case["bind"],
                        case["excl"], case["strategy"], ref=ref if case["allocated_exclusive"] else None,
                        alloc_excl=excl if case["allocated_exclusive"] else None)
    if case["want_error"]:
        assert got is None
    else:
        assert got == case["want"]


@pytest.mark.parametrize("seq", DOC["sequential"], ids=lambda s: s["name"])
def test_product_take_cpus_with_ref_counts(seq):
    topo = oracle.test_topology(*seq["topology"])
    n = len(topo[0])
    ref = np.zeros(n, np.int32)
    excl = ["" for _ in range(n)]
    for step in seq["steps"]:
        available = [c for c in range(n) if ref[c] < seq["max_ref"]]
        got = _product_take(topo, seq["max_ref"], available, step["need"], step["bind"], "None", "MostAllocated",
                            ref=ref, alloc_excl=excl)
        assert got == step["want"]
        for c in got:
            ref[c] += 1
            excl[c] = "PCPULevel"
    if "want_available_after" in seq:
        assert [c for c in range(n) if ref[c] < seq["max_ref"]] == seq["want_available_after"]
