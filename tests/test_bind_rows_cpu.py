"""NodeNUMAResource cpuset binding on nodes without a NUMA topology policy: the engine's per-pair code
(kg_row_eval, the counts the Filter's Allocate reduces to) against the oracle, which runs the reference's
Allocate literally — getAvailableCPUs, the required-policy filter, takePreferredCPUs (the CPU accumulator
pinned by cpu_accumulator_test.go) and satisfiedRequiredCPUBindPolicy — on the nodes' logical CPUs."""
import numpy as np
import pytest

from bind_cases import bind_config, make_bind_cluster
from koordinator_amd import _native as nat
from koordinator_amd import engine
from oracle import oracle


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("default", ["FullPCPUs", "SpreadByPCPUs"])
def test_bind_rows_match_oracle(seed, default):
    cl, view, idx = make_bind_cluster(40, 60, seed)
    cfg = bind_config(numa_default_cpu_bind_policy=default)
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, idx)
    assert (pods["flags"] & nat.POD_NUMA_CPU_BIND).any() and (pods["flags"] & nat.POD_NUMA_BIND_INVALID).any()
    n_ok = 0
    for i, pi in enumerate(idx):
        for j in range(len(nodes)):
            ok, score = oracle.numa_eval(cfg, view, pi, j)
            got = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], 0)
            assert (bool(got[0]), got[3] if got[0] else 0) == (bool(ok), score if ok else 0), (i, j)
            n_ok += bool(ok)
    assert 0 < n_ok < len(idx) * len(nodes)


def test_bind_counts_match_the_allocation():
    """cpuset_full_free_cpus / cpuset_free_cores are what getAvailableCPUs + the required-policy filter leave."""
    cl, view, _ = make_bind_cluster(60, 1, 7)
    cfg = bind_config()
    nodes = engine.build_node_rows(cfg, view)
    for j, n in enumerate(cl.nodes):
        if n.cpu_detail is None:
            continue
        avail = [c for c in range(len(n.cpu_detail))
                 if not (n.cpu_allocated.get(c, (0, ""))[0] >= max(n.max_ref_count, 1)) and c not in n.reserved_cpus]
        cores = {}
        for c, (_, _, core) in enumerate(n.cpu_detail):
            cores.setdefault(core, []).append(c)
        cpc = len(n.cpu_detail) // len(cores)
        full = sum(len(cs) for cs in cores.values() if all(c in avail for c in cs))
        free = sum(1 for cs in cores.values() if any(c in avail for c in cs))
        assert (nodes[j]["cpus_per_core"], nodes[j]["cpuset_full_free_cpus"], nodes[j]["cpuset_free_cores"]) == (cpc, full, free)


def test_bind_on_numa_policy_node_is_refused():
    cl, view, idx = make_bind_cluster(4, 4, 11)
    cfg = bind_config()
    n = cl.nodes[0]
    n.numa_policy, n.numa_zones, n.cpu_detail = "Restricted", [{"cpu": "4", "memory": "4Gi"}], [(0, 0, 0), (0, 0, 1)]
    n.cpu_topology_valid, n.cpu_allocated, n.reserved_cpus, n.cpu_bind_policy = True, {}, [], ""
    view = cl.view(extra_pods=[])
    from koordinator_amd.objects import Container, Pod
    pod = Pod(name="b", containers=[Container(requests={"cpu": "2"})], priority=9999,
              labels={"koordinator.sh/qosClass": "LSR"})
    view.add_pods([pod])
    prow = engine.build_pod_rows(cfg, view, [view.pod_index(pod)])
    assert prow["flags"][0] & nat.POD_NUMA_CPU_BIND
    with pytest.raises(engine.EngineError):
        engine.row_eval(cfg, engine.build_node_rows(cfg, view)[0:1], prow, 0)
