"""NodeNUMAResource cpuset binding: the engine's per-pair code (kg_row_eval, the counts the Filter's
Allocate reduces to — node-wide without a NUMA topology policy, zone by zone with one) against the oracle,
which runs the reference's Allocate literally — getAvailableCPUs, the required-policy filter, takePreferredCPUs (the CPU accumulator
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


@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_bind_on_numa_policy_nodes_match_oracle(seed):
    """Cpusets on nodes with a NUMA topology policy (FilterByNUMANode with the cpuset options: hints over
    the zones' cpu trimmed to their available CPUs for a required policy, Admit, allocateResourcesByHint,
    then allocateCPUSet zone by zone through the accumulator; Score with the node's cpuset CPUs as the
    requested cpu) — every pair against the oracle, both outcomes present."""
    cl, view, idx = make_bind_cluster(30, 50, seed, numa_frac=1.0)
    cfg = bind_config(numa_default_cpu_bind_policy="FullPCPUs" if seed % 2 else "SpreadByPCPUs")
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, idx)
    zoned = (nodes["numa_policy"] != nat.NUMA_NONE) & (nodes["n_zones"] > 0)
    bound = (pods["flags"] & nat.POD_NUMA_CPU_BIND) != 0
    seen = [0, 0]
    for i, pi in enumerate(idx):
        for j in range(len(nodes)):
            ok, score = oracle.numa_eval(cfg, view, pi, j)
            got = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], 0)
            assert (bool(got[0]), got[3] if got[0] else 0) == (bool(ok), score if ok else 0), (i, j)
            if zoned[j] and bound[i]:
                seen[bool(ok)] += 1
    assert seen[0] > 0 and seen[1] > 0, seen


def test_bind_zone_counts_match_the_allocation():
    """zone_cpus_avail / zone_cpus_full / zone_cores_free: the available CPUs of each zone's NUMA node,
    before and after each required policy's filter (trimNUMANodeResources, allocateCPUSet)."""
    cl, view, _ = make_bind_cluster(60, 1, 8, numa_frac=1.0)
    nodes = engine.build_node_rows(bind_config(), view)
    checked = 0
    for j, n in enumerate(cl.nodes):
        if n.cpu_detail is None or not n.numa_zones:
            continue
        avail = [c for c in range(len(n.cpu_detail))
                 if not (n.cpu_allocated.get(c, (0, ""))[0] >= max(n.max_ref_count, 1)) and c not in n.reserved_cpus]
        cores = {}
        for c, (_, _, core) in enumerate(n.cpu_detail):
            cores.setdefault(core, []).append(c)
        cpc = len(n.cpu_detail) // len(cores)
        assert nodes[j]["cpuset_avail_cpus"] == len(avail)
        for z, zid in enumerate(n.numa_zone_ids):
            zc = {k: cs for k, cs in cores.items() if n.cpu_detail[cs[0]][1] == zid}
            want = (sum(1 for c in avail if n.cpu_detail[c][1] == zid),
                    sum(len(cs) for cs in zc.values() if all(c in avail for c in cs) and len(cs) == cpc),
                    sum(1 for cs in zc.values() if any(c in avail for c in cs)))
            got = (nodes[j]["zone_cpus_avail"][z], nodes[j]["zone_cpus_full"][z], nodes[j]["zone_cores_free"][z])
            assert got == want, (j, z)
            checked += 1
    assert checked > 10


def test_bind_reserve_is_refused():
    """kg_row_commit of a cpuset-bound pod: choosing the CPUs (the accumulator at Reserve) is not on the
    engine path, on nodes with or without a NUMA topology policy."""
    cl, view, idx = make_bind_cluster(6, 20, 12, numa_frac=0.5)
    cfg = bind_config()
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, idx)
    i = int(np.flatnonzero(pods["flags"] & nat.POD_NUMA_CPU_BIND)[0])
    j = int(np.flatnonzero(nodes["flags"] & nat.NODE_NUMA_TOPO_VALID)[0])
    with pytest.raises(engine.EngineError):
        engine.row_commit(cfg, nodes[j:j + 1], pods[i:i + 1])
