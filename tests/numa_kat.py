"""Build clusters for the transcribed NodeNUMAResource known-answer tests (tests/golden/numa_*.json)."""
from kat import load
from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Container, Node, Pod, parse_quantity, quantity_value

NAMES = {None: None}


def numa_score_cluster(case):
    cl = Cluster()
    existing = {}
    for e in case["existing"]:
        existing.setdefault(e["node"], []).append(e)
    for nd in case["nodes"]:
        count = nd["zones"]
        cpu_m = quantity_value("cpu", nd["cpu"])
        mem = quantity_value("memory", nd["memory"])
        zone = {"cpu": f"{cpu_m // count}m", "memory": str(mem // count)}
        alloc0 = {}
        pods = []
        for e in existing.get(nd["name"], []):
            pods.append(Pod(name=f"e-{len(pods)}-{nd['name']}", containers=[Container(requests={"cpu": e["cpu"], "memory": e["memory"]})]))
            for k in ("cpu", "memory"):
                alloc0[k] = alloc0.get(k, 0) + quantity_value(k, e[k])
        node = Node(nd["name"], allocatable={"cpu": nd["cpu"], "memory": nd["memory"]}, numa_policy=nd["policy"],
                    numa_zones=[dict(zone) for _ in range(count)],
                    numa_allocated={0: {"cpu": f"{alloc0['cpu']}m", "memory": str(alloc0["memory"])}} if alloc0 else None)
        cl.add_node_with_pods(node, pods)
    pod = Pod(name="p", containers=[Container(requests=dict(case["pod"]))])
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",), numa_strategy=case["strategy"])
    return cfg, view, view.pod_index(pod), cl


def merge_lists(providers):
    """providers of a policy_test.go case → the provider lists of filterProvidersHints."""
    lists = []
    for prov in providers:
        if not prov:
            lists.append(None)               # provider without hints: one preferred any-NUMA hint
            continue
        for res, hints in prov.items():
            lists.append(None if hints is None else [(h[0], h[1]) for h in hints])
    return lists


def _amplify(x, ratio):
    """extension.Amplify (apis/extension/node_resource_amplification.go:170-175)."""
    import math
    return x if ratio <= 1 else int(math.ceil(float(x) * float(ratio)))


def _amp_pod(name, req, cpuset):
    # makePodOnNode (plugin_test.go:122-135): prod priority; a cpuset pod is LSR
    labels = {"koordinator.sh/qosClass": "LSR"} if cpuset else {}
    return Pod(name=name, containers=[Container(requests=dict(req))], priority=9999, labels=labels)


def _amp_node(name, cpu, memory, ratio, nrt, cpuset_cpus):
    """makeNode (plugin_test.go:114-120) and, for nrt nodes, the TopologyOptions the KATs install:
    buildCPUTopologyForTest(2, 1, 8, 2) — CPUs 0-15 in NUMA node 0, 16-31 in node 1 — with zones of
    Amplify(16, ratio) cpus and 20Gi; an existing cpuset pod holds CPUs 0..n-1."""
    cpu_m = _amplify(quantity_value("cpu", cpu), ratio)
    node = Node(name, allocatable={"cpu": f"{cpu_m}m", "memory": memory}, cpu_amplification_ratio=ratio)
    if nrt:
        zone = {"cpu": str(_amplify(16, ratio)), "memory": "20Gi"}
        node.numa_zones = [dict(zone), dict(zone)]
        node.cpu_topology_valid = True
        # the CPU detail of buildCPUTopologyForTest(2, 1, 8, 2): socket = NUMA node = cpu // 16, core = cpu // 2
        node.cpu_detail = [(c // 16, c // 16, c // 2) for c in range(32)]
        node.cpu_allocated = {c: (1, "PCPULevel") for c in range(cpuset_cpus)}
    return node


def amplified_score_cluster(case):
    cl = Cluster()
    for nd in case["nodes"]:
        ex = [e for e in case["existing"] if e["node"] == nd["name"]]
        cs = sum(quantity_value("cpu", e["cpu"]) // 1000 for e in ex if e["cpuset"])
        pods = [_amp_pod(f"e{i}-{nd['name']}", {"cpu": e["cpu"], "memory": e["memory"]}, e["cpuset"])
                for i, e in enumerate(ex)]
        cl.add_node_with_pods(_amp_node(nd["name"], nd["cpu"], nd["memory"], nd["ratio"], nd["nrt"], cs), pods)
    pod = _amp_pod("p", case["pod"], case["pod_cpuset"])
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",), numa_strategy=case["strategy"])
    return cfg, view, view.pod_index(pod), cl


def amplified_filter_cluster(case):
    """TestFilterWithAmplifiedCPUs: one node of cpuTopology.NumCPUs (32) cpus and 40Gi."""
    cl = Cluster()
    cs = sum(quantity_value("cpu", e["cpu"]) // 1000 for e in case["existing"] if e["cpuset"])
    pods = [_amp_pod(f"e{i}", {"cpu": e["cpu"]}, e["cpuset"]) for i, e in enumerate(case["existing"])]
    cl.add_node_with_pods(_amp_node("node-1", "32", "40Gi", case["ratio"], case["nrt"], cs), pods)
    pod = _amp_pod("p", case["pod"], case["pod_cpuset"]) if case["pod"] else Pod(name="p")
    view = cl.view(extra_pods=[pod])
    cfg = make_config(plugins=("NodeNUMAResource",))
    return cfg, view, view.pod_index(pod), cl
