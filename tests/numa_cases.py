"""Config-3 clusters with the NodeNUMAResource edge cases the plain synthetic mix does not reach.

Starts from synth.make_numa_cluster and perturbs it, seeded:

nodes
  * all four policies, BestEffort included (the only policy that runs the full non-preferred merge)
  * zone affinity ids out of list order and sparse (2·i + 1), so list order ≠ mask order
  * CPU amplification ratio 1.5 (zone cpu amplified; filterAmplifiedCPUs active)
  * zones over-allocated (available clipped at 0), zones without a memory key, no allocation entry
  * a Restricted node with no zones (Filter: node(s) missing NUMA resources)
  * invalid CPU topology (Reserve records nothing; filterAmplifiedCPUs rejects cpu requests)
  * cpuset pods on the node (whole CPUs per zone, some outside the zones): amplified node / zone cpu
  * an amplification annotation without NodeResourceTopology (nil CPU topology, no zones)
pods
  * large requests spanning several zones (minimum affinity > 1, SingleNUMANode rejects)
  * memory-only and cpu-only pods, a present-but-zero cpu key (hint list over every mask)
  * requests no zone combination can hold (empty hint list: BestEffort admits, others reject)
"""
import numpy as np

from koordinator_amd import _native as nat
from koordinator_amd import synth

MI = 1 << 20


def make_numa_edge_cluster(n_nodes: int, n_pods: int, seed: int):
    cl = synth.make_numa_cluster(n_nodes, n_pods, seed=seed, zones=(1, 2, 3, 4, 8))
    rng = np.random.default_rng(seed + 5)
    numa = cl.numa_arr
    nodes = cl.nodes
    numa["policy"] = rng.integers(0, 4, n_nodes)
    for j in range(n_nodes):
        Z = int(numa["n_zones"][j])
        u = rng.random()
        if u < 0.25:
            numa["zone_id"][j, :Z] = rng.permutation(Z)
        elif u < 0.4:
            numa["zone_id"][j, :Z] = 2 * np.arange(Z)[::-1] + 1
        if rng.random() < 0.15:
            numa["cpu_amplification_ratio"][j] = 1.5
        for z in range(Z):
            v = rng.random()
            tot, al = numa["zone_total"][j, z], numa["zone_allocated"][j, z]
            if v < 0.08:
                al["v"][nat.RES_CPU] = tot["v"][nat.RES_CPU] + 1000       # over-allocated
            elif v < 0.14:
                tot["present"] &= ~np.uint32(1 << nat.RES_MEMORY)          # zone without a memory key
                tot["v"][nat.RES_MEMORY] = 0
            elif v < 0.2:
                al["present"] = 0                                           # no allocation entry
                al["v"][:] = 0
        if rng.random() < 0.03:
            numa["policy"][j] = nat.NUMA_RESTRICTED
            numa["n_zones"][j] = 0
        if rng.random() < 0.1:
            numa["cpu_topology_valid"][j] = 0
        elif rng.random() < 0.3:
            # cpuset pods hold whole CPUs out of the zones' cpu allocations; amplified nodes mostly
            for z in range(int(numa["n_zones"][j])):
                al = numa["zone_allocated"][j, z]
                if al["present"] & np.uint32(1 << nat.RES_CPU):
                    numa["zone_cpuset_cpus"][j, z] = rng.integers(0, al["v"][nat.RES_CPU] // 1000 + 1)
            numa["cpuset_cpus"][j] = numa["zone_cpuset_cpus"][j].sum() + rng.integers(0, 3)
            if rng.random() < 0.6:
                numa["cpu_amplification_ratio"][j] = rng.choice([1.5, 2.0, 1.25])
        if rng.random() < 0.04:
            # amplification annotation without a NodeResourceTopology (CPUTopology nil)
            numa["policy"][j] = nat.NUMA_NONE
            numa["n_zones"][j] = 0
            numa["cpu_topology_valid"][j] = -1
            numa["cpuset_cpus"][j] = 0
            numa["zone_cpuset_cpus"][j] = 0
            numa["cpu_amplification_ratio"][j] = 2.0
    # pods: keep the LS / batch mix, then reshape some LS requests
    rq, lm = cl.containers["requests"], cl.containers["limits"]
    prng = np.random.default_rng(seed + 9)
    cpu_bit, mem_bit = np.uint32(1 << nat.RES_CPU), np.uint32(1 << nat.RES_MEMORY)
    for i in range(n_pods):
        if not (rq["present"][i] & cpu_bit):
            continue
        u = prng.random()
        for arr in (rq, lm):
            if u < 0.15:      # spans several zones
                arr["v"][i, nat.RES_CPU] = int(prng.choice([24_000, 40_000, 64_000]))
                arr["v"][i, nat.RES_MEMORY] = int(prng.choice([64, 128, 200])) * 1024 * MI
            elif u < 0.25:    # memory only
                arr["present"][i] &= ~cpu_bit
                arr["v"][i, nat.RES_CPU] = 0
            elif u < 0.32:    # cpu only
                arr["present"][i] &= ~mem_bit
                arr["v"][i, nat.RES_MEMORY] = 0
            elif u < 0.38:    # present-but-zero cpu key
                arr["v"][i, nat.RES_CPU] = 0
            elif u < 0.43:    # larger than any node
                arr["v"][i, nat.RES_CPU] = 10_000_000
    return synth.SynthView(cl.pods, cl.containers, nodes, cl.now_ns, numa)


def numa_config(**kw):
    from koordinator_amd.config import make_config

    return make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling", "NodeNUMAResource"), **kw)
