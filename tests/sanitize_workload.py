"""Workload of tests/test_sanitizers_cpu.py, run in a child process with the AddressSanitizer runtime
preloaded and the sanitizer builds of the host code (KG_SANITIZED_HOST_SO) and of the oracle
(KGO_SANITIZED_SO) loaded in place of the normal libraries.  It walks every host entry point over
edge-case clusters and checks the results against the oracle, so the sanitized code is also exercised
on the paths the parity tests cover.  Not a test module itself (no test_ prefix)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from kat import case_cluster, load  # noqa: E402
from numa_cases import make_numa_edge_cluster, numa_config  # noqa: E402
from numa_kat import amplified_filter_cluster, amplified_score_cluster  # noqa: E402
from rsv_cases import rows_matrix5  # noqa: E402
from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import make_config, shipped_profile  # noqa: E402
from oracle import oracle  # noqa: E402

import ctypes  # noqa: E402

assert os.environ.get("KG_SANITIZED_HOST_SO") and os.environ.get("KGO_SANITIZED_SO")
assert nat.lib()._name == os.environ["KG_SANITIZED_HOST_SO"] and oracle.lib()._name == os.environ["KGO_SANITIZED_SO"]
assert hasattr(ctypes.CDLL(None), "__asan_init"), "the ASan runtime is not loaded"


def pairs(cfg, cl, P, N):
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    out = np.zeros((4, P, N), np.int64)
    for i in range(P):
        for j in range(N):
            out[:, i, j] = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)
    return out


# config validation, including rejected arguments
buf = ctypes.create_string_buffer(256)
L = nat.lib()
for bad in ({"weight_fit": -1}, {"place_chunk": 5000}, {"numa_strategy": 9}):
    c = shipped_profile()
    for k, v in bad.items():
        c[k] = v
    assert L.kg_config_validate(nat.ptr(c), buf, 256) != 0

# Fit + LoadAware on a decorated cluster (assigned pods, PodsMetric, aggregated usages)
cl = synth.make_cluster(90, 20, seed=7)
cfg = shipped_profile()
got = pairs(cfg, cl, 20, 90)
m, f, la = oracle.eval_matrix(cfg, cl, np.arange(20), cl.now_ns)
assert (got[0].astype(bool) == m).all() and (got[1] == f).all() and (got[2] == la).all()
n_ref, s_ref = oracle.schedule(cfg, cl, np.arange(20), cl.now_ns)
top = oracle.eval_parallel(cfg, cl, np.arange(20), cl.now_ns, 4)
assert len(top) == 20

# LoadAware known answers through the host row builders
doc = load("loadaware_kat.json")
for key, pk in (("score_cases", "pod"), ("filter_cases", "test_pod")):
    for case in doc[key]:
        c, view, pi, kc = case_cluster(doc, case, pk)
        got = engine.row_eval(c, engine.build_node_rows(c, view), engine.build_pod_rows(c, view, [pi]), kc.now_ns)
        if key == "score_cases":
            assert got[2] == case["want"] == oracle.la_score(c, view, pi, 0, kc.now_ns)
        else:
            assert oracle.la_filter(c, view, pi, 0, kc.now_ns) == case["want"]

# NodeNUMAResource edge cases: per-pair evaluation and the sequential cycle with zone Reserve
cl = make_numa_edge_cluster(40, 24, seed=11)
cfg = numa_config(weight_numa=2)
got = pairs(cfg, cl, 24, 40)
m, f, la, nu = oracle.eval_matrix3(cfg, cl, np.arange(24), cl.now_ns)
assert (got[0].astype(bool) == m).all() and (got[3] == nu).all()
nodes = engine.build_node_rows(cfg, cl)
pods = engine.build_pod_rows(cfg, cl, np.arange(24))
for i in range(24):
    best, bj = -1, -1
    for j in range(40):
        ok, a, b, n = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)
        t = int(cfg["weight_fit"]) * a + int(cfg["weight_loadaware"]) * b + 2 * n
        if ok and t > best:
            best, bj = t, j
    if bj >= 0:
        engine.row_commit(cfg, nodes[bj:bj + 1], pods[i:i + 1])
oracle.schedule(cfg, cl, np.arange(24), cl.now_ns)
for case in load("numa_amplified_kat.json")["score_cases"]:
    c, view, pi, _ = amplified_score_cluster(case)
    engine.build_pod_rows(c, view, [pi])
    engine.build_node_rows(c, view)
for case in load("numa_amplified_kat.json")["filter_cases"]:
    c, view, pi, _ = amplified_filter_cluster(case)
    oracle.numa_eval(c, view, pi, 0)

# Reservation + NodeNUMAResource + ElasticQuota (shipped profile)
cl = synth.make_profile_cluster(60, 16, seed=9, rsv_node_frac=0.4, n_quotas=4)
cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "NodeNUMAResource"),
                      weight_numa=2)
got = rows_matrix5(cfg, cl, np.arange(16), cl.now_ns)
ref = oracle.eval_matrix5(cfg, cl, np.arange(16), cl.now_ns)
for a, b in zip(got, ref):
    assert (np.asarray(a) == np.asarray(b)).all()
cfg_all = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "NodeNUMAResource",
                                   "ElasticQuota"), weight_numa=2)
oracle.schedule2(cfg_all, cl, np.arange(16), cl.now_ns)
# ElasticQuota tree with EnableCheckParentQuota (the oracle's ancestor walks)
cl = synth.make_rsv_cluster(40, 30, seed=10, n_quotas=7, quota_ratio=0.4, quota_tree=True)
cfg_tree = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"),
                           eq_check_parent_quota=1)
assert L.kg_config_validate(nat.ptr(cfg_tree), buf, 256) == 0
oracle.schedule2(cfg_tree, cl, np.arange(30), cl.now_ns)
# cpuset binding, with and without NUMA topology policies (the oracle's accumulator and zone-wise take)
from bind_cases import bind_config, make_bind_cluster  # noqa: E402
cl, view, idx = make_bind_cluster(14, 18, 5, numa_frac=0.5)
cfg = bind_config()
nodes = engine.build_node_rows(cfg, view)
pods = engine.build_pod_rows(cfg, view, idx)
for i, pi in enumerate(idx):
    for j in range(len(nodes)):
        ok, score = oracle.numa_eval(cfg, view, pi, j)
        got = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], 0)
        assert (bool(got[0]), got[3] if got[0] else 0) == (bool(ok), score if ok else 0)

# LoadAware resourceWeights beyond cpu / memory (the exact pair path)
cl = synth.make_la_extra_cluster(40, 12, seed=6)
cfg = make_config(plugins=("NodeResourcesFit", "LoadAwareScheduling"),
                  resource_weights={"cpu": 1, "memory": 1, "ephemeral-storage": 1, "example.com/gpu": 2})
got = pairs(cfg, cl, 12, 40)
m, f, la = oracle.eval_matrix(cfg, cl, np.arange(12), cl.now_ns)
assert (got[0].astype(bool) == m).all() and (got[1] == f).all() and (got[2] == la).all()
print("sanitize workload ok")
