"""NodeNUMAResource Filter known answers with cpuset binding (TestPlugin_Filter, plugin_test.go:552-899;
tests/golden/numa_plugin_filter_kat.json) through the oracle and the engine's per-pair code (kg_row_eval),
including the two cases on a SingleNUMANode node (FilterByNUMANode for a cpuset)."""
import pytest

from kat import load
from koordinator_amd import engine
from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Container, Node, Pod
from oracle import oracle

DOC = load("numa_plugin_filter_kat.json")


def _cluster(case):
    ratio = case.get("ratio", 0.0)
    node = Node("test-node-1", allocatable={"cpu": "96", "memory": "512Gi"}, cpu_amplification_ratio=ratio,
                numa_policy=case.get("numa_policy", ""))
    node.numa_zones = [{"cpu": "8", "memory": "32Gi"}, {"cpu": "8", "memory": "32Gi"}]
    if case.get("topology") == "invalid":
        node.cpu_topology_valid = False
    else:
        node.cpu_detail = [(c // 8, c // 8, c // 2) for c in range(16)]   # buildCPUTopologyForTest(2, 1, 4, 2)
        node.cpu_allocated = {}
    node.cpu_bind_policy = "FullPCPUsOnly" if case.get("kubelet_full_pcpus_only") else case.get("node_cpu_bind", "")
    cl = Cluster()
    cl.add_node(node)
    p = case["pod"]
    req = {} if p["cpu"] is None else {"cpu": p["cpu"]}
    labels = {"koordinator.sh/qosClass": p["qos"]}
    pod = Pod(name="p", containers=[Container(requests=req, limits=req)], priority=9999, labels=labels,
              cpu_bind_required=p.get("required", ""), cpu_bind_preferred=p.get("preferred", ""))
    view = cl.view(extra_pods=[pod])
    return make_config(plugins=("NodeNUMAResource",)), view, view.pod_index(pod)


@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_numa_plugin_filter_kat(case):
    cfg, view, pi = _cluster(case)
    assert bool(oracle.numa_eval(cfg, view, pi, 0)[0]) == case["want"]
    rows = engine.build_node_rows(cfg, view)
    prow = engine.build_pod_rows(cfg, view, [pi])
    assert bool(engine.row_eval(cfg, rows, prow, 0)[0]) == case["want"]
