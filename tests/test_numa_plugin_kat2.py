"""NodeNUMAResource known answers transcribed from the reference's own tests:
* TestPlugin_PreFilter (plugin_test.go:228-550) — the pod rows' PreFilter state (kg_build_pod_rows);
* TestPlugin_Score (scoring_test.go:332-551) — the cpuset-pod node scores (kg_row_eval and the oracle);
* TestFilterWithNUMANodeScoring (plugin_test.go:1649-1877) — the affinity the Filter stores, pinned through the
  oracle's hint and the zone a Reserve allocates on (kg_row_commit).
GPU runs of the Score and NUMA-node-scoring cases are in test_numa_gpu.py; the hint lists of
TestResourceManagerGetTopologyHint (resource_manager_test.go:591-1026) pin the oracle's hint generation directly."""
import numpy as np
import pytest

from kat import load
from koordinator_amd import _native as nat
from koordinator_amd import engine
from koordinator_amd.config import make_config
from koordinator_amd.objects import CPU_BIND, Cluster, Container, Node, Pod
from oracle import oracle

PREFILTER = load("numa_prefilter_kat.json")
SCORE = load("numa_plugin_score_kat.json")
NODE_SCORING = load("numa_node_scoring_kat.json")


def _topology(s, nps, cpn, cpc):
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57)."""
    out, node, core = [], 0, 0
    for sk in range(s):
        for _ in range(nps):
            for _ in range(cpn):
                for _ in range(cpc):
                    out.append((sk, node, core))
                core += 1
            node += 1
    return out


@pytest.mark.parametrize("case", PREFILTER["cases"], ids=lambda c: c["name"])
def test_prefilter_state_kat(case):
    cl = Cluster()
    cl.add_node(Node("n", allocatable={"cpu": "96", "memory": "512Gi"}))
    req = {} if case["cpu"] is None else {"cpu": case["cpu"]}
    labels = {} if case["qos"] is None else {"koordinator.sh/qosClass": case["qos"]}
    pod = Pod(name="p", containers=[] if case.get("no_containers") else [Container(requests=req)],
              priority=case["priority"], labels=labels, cpu_bind_required=case.get("required", ""),
              cpu_bind_preferred=case.get("preferred", ""))
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",),
                      numa_default_cpu_bind_policy=case.get("default_bind", "FullPCPUs"))
    row = engine.build_pod_rows(cfg, view, [view.pod_index(pod)])[0]
    want, flags = case["want"], int(row["flags"])
    if want.get("invalid"):
        assert flags & nat.POD_NUMA_BIND_INVALID
        return
    assert not flags & nat.POD_NUMA_BIND_INVALID
    assert bool(flags & nat.POD_NUMA_SKIP) == want["skip"]
    if want["skip"]:
        return
    assert bool(flags & nat.POD_NUMA_CPU_BIND) == want["bind"]
    assert int(row["numa_request"][nat.RES_CPU]) // 1000 == want["cpus"]
    if want["bind"]:
        cb = int(row["cpu_bind"])
        assert cb & 15 == CPU_BIND[want["required"]]
        assert (cb >> 4) & 15 == CPU_BIND[want["preferred"]]


def score_cluster(case):
    cl = Cluster()
    topo = None if case["topology"] is None else _topology(*case["topology"])
    ncpu = 96 if topo is None else len(topo)
    node = Node("test-node-1", allocatable={"cpu": f"{ncpu * 1000}m", "memory": "512Gi"})
    if topo is not None:
        node.numa_zones = []
        node.cpu_detail = topo
        node.cpu_allocated = {}
    node.cpu_bind_policy = case.get("node_cpu_bind_policy", "")
    node.numa_allocate_strategy = case.get("numa_allocate_strategy", "")
    cl.add_node(node)
    req = {"cpu": str(case["cpus"])} if case["cpus"] else {}
    pod = Pod(name="p", containers=[Container(requests=req)] if req else [], priority=9999,
              labels={"koordinator.sh/qosClass": "LSR"}, cpu_bind_preferred=case["preferred"])
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",), numa_strategy="MostAllocated", numa_resources={"cpu": 1})
    return cfg, view, view.pod_index(pod)


@pytest.mark.parametrize("case", SCORE["cases"], ids=lambda c: c["name"])
def test_plugin_score_kat(case):
    cfg, view, pi = score_cluster(case)
    ok, score = oracle.numa_eval(cfg, view, pi, 0)
    assert ok and score == case["want"]
    f, _, _, numa = engine.row_eval(cfg, engine.build_node_rows(cfg, view), engine.build_pod_rows(cfg, view, [pi]), 0)
    assert f and numa == case["want"]


def node_scoring_cluster(case):
    n = case["zones"]
    node = Node("test-node-1", allocatable={"cpu": "104", "memory": "256Gi"}, numa_policy=case["policy"])
    node.numa_zones = [{"cpu": f"{104000 // n}m", "memory": str(256 * 1024 ** 3 // n)} for _ in range(n)]
    node.numa_zone_ids = list(range(n))
    alloc = {}
    for z, pods in case["existing"].items():
        cpu = sum(int(c) * 1000 for c, _ in pods)
        mem = sum(int(m[:-2]) * 1024 ** 3 for _, m in pods)
        alloc[int(z)] = {"cpu": f"{cpu}m", "memory": str(mem)}
    node.numa_allocated = alloc
    cores = 104 // 2 // n
    node.cpu_detail = _topology(n, 1, cores, 2)   # options.CPUTopology of the test (a valid topology)
    node.cpu_allocated = {}
    cl = Cluster()
    cl.add_node(node)
    pod = Pod(name="p", containers=[Container(requests={"cpu": "4", "memory": "40Gi"})])
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",), numa_hint_strategy=case["hint_strategy"])
    return cfg, view, view.pod_index(pod)


@pytest.mark.parametrize("case", NODE_SCORING["cases"], ids=lambda c: c["name"])
def test_filter_with_numa_node_scoring_kat(case):
    cfg, view, pi = node_scoring_cluster(case)
    ok, mask = oracle.numa_hint(cfg, view, pi, 0)
    assert ok and mask == 1 << case["want_zone"]
    rows = engine.build_node_rows(cfg, view)
    prow = engine.build_pod_rows(cfg, view, [pi])
    assert engine.row_eval(cfg, rows, prow, 0)[0]
    before = rows["zone_allocated"][0].copy()
    engine.row_commit(cfg, rows, prow)   # Reserve allocates on the stored hint's zone
    grew = np.flatnonzero((rows["zone_allocated"][0] != before).any(axis=1)).tolist()
    assert grew == [case["want_zone"]]


HINTS = load("numa_topology_hint_kat.json")


@pytest.mark.parametrize("case", HINTS["cases"], ids=lambda c: c["name"])
def test_resource_manager_topology_hint_kat(case):
    """The oracle's generateResourceHints (with trimNUMANodeResources for a required cpuset policy) against the
    reference's hint lists."""
    node = Node("test-node", allocatable={"cpu": "104", "memory": "256Gi"},
                cpu_amplification_ratio=float(case["ratio"]), numa_policy="Restricted")
    node.numa_zones = [{"cpu": "52", "memory": "128Gi"}, {"cpu": "52", "memory": "128Gi"}]
    node.numa_zone_ids = [0, 1]
    node.cpu_detail = _topology(2, 1, 26, 2)
    alloc = case["allocated"]
    node.cpu_allocated = {} if alloc is None else {c: (1, "None") for a, b in alloc["cpuset"] for c in range(a, b + 1)}
    if alloc is not None:
        node.numa_allocated = {int(z): {"cpu": q} for z, q in alloc["zones"].items()}
    cl = Cluster()
    cl.add_node(node)
    pod = Pod(name="p", containers=[Container(requests={"cpu": "4"})])
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",))
    lists = oracle.numa_hint_lists(cfg, view, view.pod_index(pod), 0, bind=case["bind"],
                                   required=CPU_BIND[case["required"]])
    want = [(sum(1 << b for b in bits), pref) for bits, pref in case["want_cpu"]]
    assert set(lists) == {nat.RES_CPU}
    assert lists[nat.RES_CPU] == want
