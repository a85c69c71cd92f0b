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
