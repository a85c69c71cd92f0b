"""NodeNUMAResource (config 3) on the host: the engine's per-pair code (kg_numa_pair, run on the CPU
through ``kg_row_eval``) and its Reserve (``kg_row_commit``) against the oracle restatement.

These are the same __host__ __device__ functions the HIP kernels execute (koordinator_amd/csrc/
kg_common.h); the GPU parity tests (test_parity_gpu.py) check the kernels themselves.
"""
import numpy as np
import pytest

from kat import load
from numa_cases import make_numa_edge_cluster, numa_config
from numa_kat import amplified_filter_cluster, amplified_score_cluster, numa_score_cluster
from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from oracle import oracle

SCORE = load("numa_score_kat.json")
AMP = load("numa_amplified_kat.json")

CONFIGS = {
    "least": dict(),
    "most": dict(numa_strategy="MostAllocated", numa_hint_strategy="MostAllocated", weight_numa=3,
                 numa_resources={"cpu": 2, "memory": 1}),
    "mixed": dict(numa_strategy="LeastAllocated", numa_hint_strategy="MostAllocated", weight_numa=2),
}


def _pairs(cfg, cl, P, N):
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    out = np.zeros((4, P, N), np.int64)
    for i in range(P):
        for j in range(N):
            out[:, i, j] = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)
    return out


@pytest.mark.parametrize("name", sorted(CONFIGS))
@pytest.mark.parametrize("seed", [11, 12])
def test_row_eval_matches_oracle_edge_cases(name, seed):
    P, N = 60, 90
    cl = make_numa_edge_cluster(N, P, seed=seed)
    cfg = numa_config(**CONFIGS[name])
    got = _pairs(cfg, cl, P, N)
    m, f, l, n = oracle.eval_matrix3(cfg, cl, np.arange(P), cl.now_ns)
    np.testing.assert_array_equal(got[0].astype(bool), m)
    np.testing.assert_array_equal(got[1], f)
    np.testing.assert_array_equal(got[2], l)
    np.testing.assert_array_equal(got[3], n)


def test_row_eval_matches_oracle_config3_mix():
    P, N = 50, 120
    cl = synth.make_numa_cluster(N, P, seed=3)
    cfg = numa_config()
    got = _pairs(cfg, cl, P, N)
    m, f, l, n = oracle.eval_matrix3(cfg, cl, np.arange(P), cl.now_ns)
    assert 0.2 < m.mean() < 0.95
    np.testing.assert_array_equal(got[0].astype(bool), m)
    np.testing.assert_array_equal(got[3], n)


@pytest.mark.parametrize("case", SCORE["cases"], ids=lambda c: c["name"])
def test_row_eval_numa_score_kat(case):
    """TestNUMANodeScore (nodenumaresource/scoring_test.go) through the engine's per-pair code."""
    cfg, view, pi, cl = numa_score_cluster(case)
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, [pi])
    got = [engine.row_eval(cfg, nodes[j:j + 1], pods, 0)[3]
           for j in range(len(case["nodes"]))]
    assert got == case["want"]


@pytest.mark.parametrize("seed", [21, 22])
def test_row_commit_numa_matches_sequential_oracle(seed):
    """Sequential cycle over host rows (kg_row_eval + kg_row_commit with zone allocations) == the
    oracle's kgo_schedule (NodeNUMAResource Reserve included)."""
    P, N = 70, 40
    cl = make_numa_edge_cluster(N, P, seed=seed)
    cfg = numa_config(weight_numa=2)
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    wf, wl, wn = int(cfg["weight_fit"]), int(cfg["weight_loadaware"]), int(cfg["weight_numa"])
    got_n, got_s = [], []
    for i in range(P):
        best, bj = -1, -1
        for j in range(N):
            ok, f, l, n = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)
            t = wf * f + wl * l + wn * n
            if ok and t > best:
                best, bj = t, j
        got_n.append(bj)
        got_s.append(best)
        if bj >= 0:
            engine.row_commit(cfg, nodes[bj:bj + 1], pods[i:i + 1])
    ref_n, ref_s = oracle.schedule(cfg, cl, np.arange(P), cl.now_ns)
    np.testing.assert_array_equal(np.array(got_n), ref_n)
    np.testing.assert_array_equal(np.array(got_s), ref_s)
    assert (nodes["zone_allocated"] != engine.build_node_rows(cfg, cl)["zone_allocated"]).any()


@pytest.mark.parametrize("case", AMP["score_cases"], ids=lambda c: c["name"])
def test_row_eval_amplified_score_kat(case):
    """TestScoreWithAmplifiedCPUs through the engine's per-pair code, cpuset pods (LSR prod, integer cpus,
    the default FullPCPUs policy: requestCPUBind) included."""
    cfg, view, pi, cl = amplified_score_cluster(case)
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, [pi])
    assert bool(pods["flags"][0] & nat.POD_NUMA_CPU_BIND) == case["pod_cpuset"]
    got = [engine.row_eval(cfg, nodes[j:j + 1], pods, 0) for j in range(len(case["nodes"]))]
    assert all(g[0] for g in got)
    assert [g[3] for g in got] == case["want"]


@pytest.mark.parametrize("case", AMP["filter_cases"], ids=lambda c: c["name"])
def test_row_eval_amplified_filter_kat(case):
    cfg, view, pi, cl = amplified_filter_cluster(case)
    nodes = engine.build_node_rows(cfg, view)
    pods = engine.build_pod_rows(cfg, view, [pi])
    assert bool(pods["flags"][0] & nat.POD_NUMA_CPU_BIND) == case["pod_cpuset"]
    assert bool(engine.row_eval(cfg, nodes, pods, 0)[0]) == case["want"]


def test_edge_cases_reach_the_cpuset_terms():
    """The edge clusters exercise the amplified cpuset terms: zeroing the cpuset counts changes some
    feasibility bits and some scores."""
    P, N = 60, 200
    cl = make_numa_edge_cluster(N, P, seed=13)
    cfg = numa_config()
    m, f, l, n = oracle.eval_matrix3(cfg, cl, np.arange(P), cl.now_ns)
    numa = cl.numa_arr.copy()
    numa["cpuset_cpus"] = 0
    numa["zone_cpuset_cpus"] = 0
    bare = synth.SynthView(cl.pods, cl.containers, cl.nodes, cl.now_ns, numa)
    m0, f0, l0, n0 = oracle.eval_matrix3(cfg, bare, np.arange(P), cl.now_ns)
    assert (m != m0).any()
    assert (n != n0).any()
    assert (cl.numa_arr["cpu_topology_valid"] == -1).any()
