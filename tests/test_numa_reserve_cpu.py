"""NodeNUMAResource cpuset Reserve on the CPU: TestPlugin_Reserve (plugin_test.go:1014-1151) through the engine's
host Reserve (kg_row_reserve) and the oracle's literal cycle, and randomized cpuset-binding clusters placed by a
host cycle over the engine's per-pair code (kg_row_eval + kg_row_reserve) against the oracle."""
import json
import os

import numpy as np
import pytest

from bind_cases import make_bind_cluster
from koordinator_amd import _native as nat
from koordinator_amd import engine
from koordinator_amd.config import make_config, shipped_profile
from koordinator_amd.objects import Cluster, Container, Node, Pod
from oracle import oracle
from reserve_cycle import cpu_tables, host_cycle

DOC = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "numa_reserve_kat.json")))


def _topology(s, nps, cpn, cpc):
    """buildCPUTopologyForTest (cpu_accumulator_test.go:30-57): (socket, node, core) per cpu id."""
    out, node, core = [], 0, 0
    for sk in range(s):
        for _ in range(nps):
            for _ in range(cpn):
                for _ in range(cpc):
                    out.append((sk, node, core))
                core += 1
            node += 1
    return out


def _case_cluster(case):
    cl = Cluster()
    node = Node("test-node-1", allocatable={"cpu": "96", "memory": "512Gi"})
    if case["topology"] is not None:
        node.numa_zones = []
        node.cpu_detail = _topology(*case["topology"])
        node.cpu_allocated = {c: (1, "None") for c in case.get("allocated", [])}
    elif case.get("topology_invalid"):
        node.numa_zones = []
        node.cpu_topology_valid = False
    node.cpu_bind_policy = case.get("node_cpu_bind_policy", "")
    node.numa_allocate_strategy = case.get("numa_allocate_strategy", "")
    cl.add_node(node)
    pc = case["pod"]
    req = {}
    if pc.get("cpu"):
        req["cpu"] = pc["cpu"]
    if pc.get("batch_cpu"):
        req["kubernetes.io/batch-cpu"] = pc["batch_cpu"]
    pod = Pod(name="p", containers=[Container(requests=req, limits=req)],
              priority=9999 if pc["qos"] != "BE" else 5000, labels={"koordinator.sh/qosClass": pc["qos"]},
              cpu_bind_preferred=pc.get("preferred", ""))
    view = cl.view(extra_pods=[pod])
    return view, view.pod_index(pod)


def _cfg():
    return make_config(plugins=("NodeNUMAResource",))


@pytest.mark.parametrize("case", DOC["cases"], ids=[c["name"] for c in DOC["cases"]])
def test_plugin_reserve_kat_host(case):
    view, pi = _case_cluster(case)
    cfg = _cfg()
    row = engine.build_node_rows(cfg, view)
    pod = engine.build_pod_rows(cfg, view, [pi])
    tabs = cpu_tables(view)
    if 0 in tabs:
        first, n, max_ref, strat = tabs[0]
        cpus = view.cpu_arr[first:first + n].copy()
    else:
        max_ref, strat, cpus = 1, 0, np.zeros(0, nat.CPU_INFO)
    before = row.copy()
    taken = engine.row_reserve(cfg, row, pod, cpus, max_ref, strat)
    if case["want"] == "fail":
        assert taken is None
        assert row.tobytes() == before.tobytes()   # a failed Reserve changes nothing
        return
    assert taken is not None
    assert sorted(np.flatnonzero(taken).tolist()) == case["want_cpuset"]
    if case["want_cpuset"]:
        assert (cpus["refcount"][taken] == view.cpu_arr[tabs[0][0]:][:len(cpus)]["refcount"][taken] + 1).all()
        # the row's counts follow the table (what kg_build_node_rows would derive from it)
        assert int(row["cpuset_milli"][0]) == 1000 * int((cpus["refcount"] > 0).sum())


@pytest.mark.parametrize("case", [c for c in DOC["cases"] if c["topology"] is not None],
                         ids=[c["name"] for c in DOC["cases"] if c["topology"] is not None])
def test_plugin_reserve_kat_oracle(case):
    """The oracle's cycle (Filter, then Reserve) on the one-node cluster: the cpuset it records."""
    view, pi = _case_cluster(case)
    nodes, _, cpus = oracle.schedule_cpus(_cfg(), view, [pi], 0)
    got = sorted(np.flatnonzero(cpus["refcount"] - view.cpu_arr["refcount"]).tolist())
    if case["want"] == "fail":
        assert nodes[0] == -1 and got == []
    else:
        assert nodes[0] == 0 and got == case["want_cpuset"]


@pytest.mark.parametrize("seed,n_nodes,n_pods,numa_frac", [(11, 40, 60, 0.35), (12, 24, 80, 1.0), (13, 60, 40, 0.0)])
def test_host_cycle_matches_oracle(seed, n_nodes, n_pods, numa_frac):
    """Sequential placement with cpuset Reserve: the engine's host per-pair code vs the oracle's cycle —
    placements, scores and every node's CPUs after the last Reserve."""
    cl, view, idx = make_bind_cluster(n_nodes, n_pods, seed, numa_frac=numa_frac)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    nodes, scores, rows, cpus = host_cycle(cfg, view, idx, cl.now_ns)
    ref_nodes, ref_scores, ref_cpus = oracle.schedule_cpus(cfg, view, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(cpus, ref_cpus)
    bound = int((cpus["refcount"] != view.cpu_arr["refcount"]).sum())
    assert bound > 0 and (nodes >= 0).sum() > n_pods // 4


def test_reserve_failure_after_filter():
    """A failed Reserve places nothing and changes nothing; later pods are placed as if it never happened."""
    from bind_cases import make_reserve_fail_cluster
    cl, view, idx = make_reserve_fail_cluster()
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    nodes, scores, rows, cpus = host_cycle(cfg, view, idx, cl.now_ns)
    ref_nodes, ref_scores, ref_cpus = oracle.schedule_cpus(cfg, view, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(cpus, ref_cpus)
    assert nodes.tolist() == [-1, 0, 0]
    assert np.flatnonzero(cpus["refcount"][:8]).tolist() == [2, 3, 4, 5, 6, 7]
