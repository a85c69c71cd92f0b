"""Seeded clusters for NodeNUMAResource cpuset binding: nodes with
reported CPU topologies (1–2 sockets, 1–2 NUMA nodes per socket, 2–8 cores per NUMA node, 1–2 threads
per core; some with sparse core ids socket << 16 | core), a NUMA topology policy on some of them (one zone
per NUMA node, zone allocations), node allocations (refcounts up to MaxRefCount,
exclusive policies), reserved CPUs, node CPU bind policies, cpu amplification ratios, invalid / missing
topologies; pods that bind cpusets (LSE / LSR prod, required / preferred / default / exclusive policies,
whole and fractional cpu requests) and pods that a node's CPU bind policy binds."""
import numpy as np

from koordinator_amd.config import make_config
from koordinator_amd.objects import Cluster, Container, Node, Pod

BIND = ["", "", "Default", "FullPCPUs", "SpreadByPCPUs", "ConstrainedBurst"]
EXCL = ["", "None", "PCPULevel", "NUMANodeLevel"]
NODE_BIND = ["", "", "", "None", "FullPCPUsOnly", "SpreadByPCPUs"]


def _topology(rng):
    s, nps, cpn, tpc = rng.choice([1, 2]), rng.choice([1, 2]), rng.choice([2, 4, 8]), rng.choice([1, 2])
    sparse = rng.random() < 0.3
    out, node_id, core_id = [], 0, 0
    for sk in range(s):
        for _ in range(nps):
            for _ in range(cpn):
                for _ in range(tpc):
                    out.append((int(sk), node_id, (sk << 16 | core_id) if sparse else core_id))
                core_id += 1
            node_id += 1
    return out


def make_bind_cluster(n_nodes: int, n_pods: int, seed: int, numa_frac: float = 0.35):
    rng = np.random.default_rng(seed)
    cl = Cluster()
    for j in range(n_nodes):
        detail = _topology(rng)
        ncpu = len(detail)
        kind = rng.random()
        ratio = float(rng.choice([0.0, 1.0, 1.5, 2.0]))
        alloc_cpu = int(np.ceil(ncpu * 1000 * ratio)) if ratio > 1 else ncpu * 1000
        node = Node(f"n{j}", allocatable={"cpu": f"{alloc_cpu}m", "memory": f"{ncpu * 4}Gi"},
                    cpu_amplification_ratio=ratio)
        held = 0
        if kind < 0.85:   # a reported topology with its node allocation
            node.numa_zones = []
            node.cpu_detail = detail
            node.max_ref_count = int(rng.choice([1, 1, 2]))
            alloc = {}
            for c in rng.choice(ncpu, size=int(rng.integers(0, ncpu + 1)), replace=False):
                alloc[int(c)] = (int(rng.integers(1, node.max_ref_count + 1)), str(rng.choice(EXCL[1:])))
            node.cpu_allocated = alloc
            held = len(alloc)
            node.reserved_cpus = [int(c) for c in rng.choice(ncpu, size=int(rng.integers(0, 3)), replace=False)]
            node.cpu_bind_policy = str(rng.choice(NODE_BIND))
            if rng.random() < numa_frac:   # a NUMA topology policy: one zone per NUMA node of the detail
                node.numa_policy = str(rng.choice(["BestEffort", "Restricted", "SingleNUMANode"]))
                ids = sorted({nd for _, nd, _ in detail})
                per = {i: sum(1 for _, nd, _ in detail if nd == i) for i in ids}
                node.numa_zones = [{"cpu": f"{per[i]}", "memory": f"{per[i] * 4}Gi"} for i in ids]
                node.numa_zone_ids = ids
                zheld = {i: sum(1 for c in alloc if detail[c][1] == i) for i in ids}
                node.numa_allocated = {i: {"cpu": f"{zheld[i] * 1000 + int(rng.integers(0, 2)) * 500}m",
                                           "memory": f"{int(rng.integers(0, per[i] * 3))}Gi"}
                                       for i in ids if rng.random() < 0.8}
        elif kind < 0.93:  # reported but invalid topology
            node.numa_zones = []
            node.cpu_topology_valid = False
        # else: no NodeResourceTopology (nil topology)
        req_cpu = held * 1000 + int(rng.integers(0, max(1, alloc_cpu - held * 1000)))
        cl.add_node(node, requested={"cpu": f"{req_cpu}m", "memory": f"{int(rng.integers(0, ncpu * 2))}Gi"},
                    pod_count=int(rng.integers(0, 20)))
    pods = []
    for i in range(n_pods):
        u = rng.random()
        cores = int(rng.choice([1, 2, 3, 4, 6, 8, 12]))
        cpu = f"{cores}" if rng.random() < 0.85 else f"{cores * 1000 + 500}m"
        req = {"cpu": cpu, "memory": f"{int(rng.integers(1, 8))}Gi"}
        if u < 0.6:       # AllowUseCPUSet pods
            p = Pod(name=f"p{i}", containers=[Container(requests=req, limits=req)], priority=9999,
                    labels={"koordinator.sh/qosClass": str(rng.choice(["LSR", "LSE"]))},
                    cpu_bind_required=str(rng.choice(BIND)), cpu_bind_preferred=str(rng.choice(BIND)),
                    cpu_exclusive=str(rng.choice(EXCL)))
        elif u < 0.95:    # LS prod: a node CPU bind policy binds it
            p = Pod(name=f"p{i}", containers=[Container(requests=req)], priority=9999)
        else:             # no requests: PreFilter skip
            p = Pod(name=f"p{i}", containers=[Container()], priority=9999)
        pods.append(p)
    view = cl.view(extra_pods=pods)
    return cl, view, [view.pod_index(p) for p in pods]


def bind_config(**kw):
    return make_config(plugins=("NodeNUMAResource",), **kw)


def make_reserve_fail_cluster():
    """A Reserve that fails after the Filter passed (resource_manager.go:296-299 "not enough cpus available to
    satisfy request"): node n0 has 8 logical CPUs, 2 of them reserved, and 8 cpu allocatable; a pod preferring
    FullPCPUs for 8 CPUs passes Fit and the Filter (no required policy, no NUMA topology policy: no Allocate
    there), its Reserve finds 6 available CPUs and fails, and the next pods still land on the node."""
    cl = Cluster()
    node = Node("n0", allocatable={"cpu": "8", "memory": "32Gi"})
    node.numa_zones = []
    node.cpu_detail = [(0, 0, c // 2) for c in range(8)]
    node.cpu_allocated = {}
    node.reserved_cpus = [0, 1]
    cl.add_node(node, requested={"cpu": "0", "memory": "0"})
    cl.add_node(Node("n1", allocatable={"cpu": "1", "memory": "32Gi"}))   # too small for any of the pods
    pods = []
    for i, cpu in enumerate(["8", "2", "4"]):
        req = {"cpu": cpu, "memory": "1Gi"}
        pods.append(Pod(name=f"p{i}", containers=[Container(requests=req, limits=req)], priority=9999,
                        labels={"koordinator.sh/qosClass": "LSR"}, cpu_bind_preferred="FullPCPUs"))
    view = cl.view(extra_pods=pods)
    return cl, view, [view.pod_index(p) for p in pods]
