"""Parity at the sizes BASELINE.json's configs are benchmarked at (SURVEY §8d gate 1: the planes on a
pod sample at full scale, the placements on the sequential cycle), on the bench's own seeded clusters.

* config 2 — 10k pods × 100k nodes (seed 2, shipped profile): the top-1 of every pod against the
  oracle's Parallelizer-faithful evaluation; mask and both score planes of every pod (all 1e9 pairs) through
  the pods' raw-spec groups, and of a 128-pod sample directly;
* config 3 — NodeNUMAResource over 100k nodes with 4/6/8 zones, 1k pods: the four planes of every pod
  through its raw-spec group, and the planes and top-1 of a 32-pod sample;
* config 5's matrix section — 1k pods × 100k nodes, 15k reservations, 64 quota groups: every plane and top-1
  of every pod;
* config 4's shape on one GPU — 1M nodes: the top-1 of 16 pods (matrix mode without planes);
* config 5 — 100k batch pods × 100k nodes with Reservation + ElasticQuota: kg_place of the first 256
  pods against the oracle's sequential cycle, with the reservation and quota state afterwards.

The clusters carry the decorated node-side LoadAware inputs (synth.decorate: assigned pods, PodsMetric,
aggregated usages, NonZeroRequested ≠ Requested, annotations).  The oracle samples run in threads
(ctypes releases the GIL; the oracle keeps per-thread scratch only).
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu

WORKERS = min(16, os.cpu_count() or 1)


def _sample(P, k, seed):
    return np.sort(np.random.default_rng(seed).choice(P, size=min(k, P), replace=False))


def _oracle_rows(fn, pods):
    """fn(one-pod index array) → tuple of [1][N] planes, run over `pods` in threads; rows stacked."""
    with ThreadPoolExecutor(WORKERS) as ex:
        parts = list(ex.map(lambda p: fn(np.array([p])), pods))
    return [np.concatenate([p[i] for p in parts]) for i in range(len(parts[0]))]


def _top1_parallel(cfg, cl, idx):
    return oracle.eval_parallel(cfg, cl, idx, cl.now_ns, WORKERS)


def spec_groups(cl, P):
    """The pending pods [0, P) grouped by their raw spec (the pod record without its identity and container
    offsets, plus its containers' and init containers' requests / limits): pods of one group are the same pod
    to every plugin, so the reference answers them with the same rows.  Returns {representative: members}."""
    pods = cl.pods[:P].copy()
    for f in ("name_id", "first_container", "first_init_container"):
        pods[f] = 0
    cont = cl.containers
    groups = {}
    for i in range(P):
        p = cl.pods[i]
        c0, ci = int(p["first_container"]), int(p["first_init_container"])
        key = (pods[i].tobytes() + cont[c0:c0 + int(p["n_containers"])].tobytes() +
               cont[ci:ci + int(p["n_init_containers"])].tobytes())
        groups.setdefault(key, []).append(i)
    return {g[0]: np.array(g) for g in groups.values()}


def check_planes_by_group(groups, oracle_rows, res, N, planes):
    """Every pod's planes against the oracle's rows of its group's representative (all P × N pairs).
    planes: names of the arrays oracle_rows returns after the mask, each paired with a slice of res."""
    reps = np.array(sorted(groups))
    ref = oracle_rows(reps)
    for k, r in enumerate(reps):
        mem = groups[r]
        for j in range(0, len(mem), 256):
            part = mem[j:j + 256]
            np.testing.assert_array_equal(engine.unpack_mask(res["mask"][part], N), np.broadcast_to(ref[0][k], (len(part), N)))
            for q, get in enumerate(planes):
                np.testing.assert_array_equal(get(res, part)[:, :N], np.broadcast_to(ref[q + 1][k], (len(part), N)))
    return ref, reps


@pytest.fixture(scope="module")
def config2():
    P, N = synth.CONFIGS[2]["n_pods"], synth.CONFIGS[2]["n_nodes"]
    cl = synth.make_cluster(N, P, seed=2)
    cfg = shipped_profile()
    eng = engine.Engine(cfg)
    eng.load_snapshot(engine.build_node_rows(cfg, cl))
    eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
    res = eng.eval(cl.now_ns)
    eng.close()
    return cfg, cl, res


def test_config2_top1_every_pod(config2):
    cfg, cl, res = config2
    want = _top1_parallel(cfg, cl, np.arange(len(res["top1"])))
    np.testing.assert_array_equal(res["top1"], want)
    assert (want != 0).mean() > 0.9


def test_config2_planes_every_pod(config2):
    """All 10k × 100k pairs: the pods' raw specs form ~105 groups; each pod's mask and both score planes
    equal the oracle's rows of its group."""
    cfg, cl, res = config2
    N, P = len(cl.nodes), len(res["top1"])
    groups = spec_groups(cl, P)
    assert len(groups) < P
    check_planes_by_group(groups, lambda reps: _oracle_rows(lambda i: oracle.eval_matrix(cfg, cl, i, cl.now_ns), reps),
                          res, N, [lambda r, q: r["scores"][q, :, 0], lambda r, q: r["scores"][q, :, 1]])


def test_config2_planes_pod_sample(config2):
    cfg, cl, res = config2
    N = len(cl.nodes)
    pods = _sample(len(res["top1"]), 128, 202)
    m, fit, la = _oracle_rows(lambda i: oracle.eval_matrix(cfg, cl, i, cl.now_ns), pods)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"][pods], N), m)
    np.testing.assert_array_equal(res["scores"][pods, :N, 0], fit)
    np.testing.assert_array_equal(res["scores"][pods, :N, 1], la)
    assert 0.1 < m.mean() < 0.95


def test_config3_pod_sample():
    P, N = 1_000, 100_000
    cl = synth.make_numa_cluster(N, P, seed=3)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
        res = eng.eval(cl.now_ns)
    # every pod through its raw-spec group (~70 groups), then a direct sample
    check_planes_by_group(spec_groups(cl, P),
                          lambda reps: _oracle_rows(lambda i: oracle.eval_matrix3(cfg, cl, i, cl.now_ns), reps), res, N,
                          [lambda r, q: r["scores"][q, :, 0], lambda r, q: r["scores"][q, :, 1],
                           lambda r, q: r["numa_scores"][q]])
    pods = _sample(P, 32, 303)
    m, f, l, n = _oracle_rows(lambda i: oracle.eval_matrix3(cfg, cl, i, cl.now_ns), pods)
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"][pods], N), m)
    np.testing.assert_array_equal(res["scores"][pods, :N, 0], f)
    np.testing.assert_array_equal(res["scores"][pods, :N, 1], l)
    np.testing.assert_array_equal(res["numa_scores"][pods, :N], n)
    tot = np.where(m, f.astype(np.int64) + l.astype(np.int64) + int(cfg["weight_numa"]) * n.astype(np.int64), -1)
    node, best = engine.decode_top1(res["top1"][pods])
    np.testing.assert_array_equal(node, np.where(tot.max(axis=1) >= 0, tot.argmax(axis=1), -1))
    np.testing.assert_array_equal(best, tot.max(axis=1))


def test_config4_million_nodes_top1():
    N, P = synth.CONFIGS[4]["n_nodes"], 16
    cl = synth.make_cluster(N, P, seed=4)
    cfg = shipped_profile()
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
        res = eng.eval(cl.now_ns, mask=False, scores=False)
    np.testing.assert_array_equal(res["top1"], _top1_parallel(cfg, cl, np.arange(P)))


def test_config5_matrix_every_pod():
    """The bench's config-5 matrix section at its size: 1,000 batch pods × 100k nodes with 15k reservations on
    10k nodes and 64 ElasticQuota groups; mask, Fit / LoadAware / Reservation planes and top-1 of every pod against
    the oracle (oracle/koord_oracle.c kgo_eval5: restore, Reservation.Filter, scoreReservation, NormalizeScore)."""
    N, P = 100_000, 1_000
    cl = synth.make_rsv_cluster(N, P, seed=5)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_RESERVATION | nat.PLUGIN_ELASTICQUOTA
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
        res = eng.eval(cl.now_ns)
    m, fit, la, _, rsv, top1 = _oracle_rows(lambda i: oracle.eval_matrix5(cfg, cl, i, cl.now_ns), np.arange(P))
    np.testing.assert_array_equal(engine.unpack_mask(res["mask"], N), m)
    np.testing.assert_array_equal(res["scores"][:, :N, 0], fit)
    np.testing.assert_array_equal(res["scores"][:, :N, 1], la)
    np.testing.assert_array_equal(res["rsv_scores"][:, :N], rsv)
    np.testing.assert_array_equal(res["top1"], top1)
    assert rsv.max() == 100 and m.mean() > 0.05


def test_config5_first_pods_placement():
    N, P, K = 100_000, 100_000, 256
    cl = synth.make_rsv_cluster(N, P, seed=5)
    cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"))
    idx = np.arange(K)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        rsv_after = eng.download_reservations()
        q_after = eng.download_quotas()
    ref_nodes, ref_scores, ref_rsv, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_nodes)
    np.testing.assert_array_equal(scores, ref_scores)
    np.testing.assert_array_equal(rsv_after["n_assigned"], ref_rsv["n_assigned"])
    np.testing.assert_array_equal(rsv_after["allocated"]["v"], ref_rsv["allocated"]["v"])
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    rnodes = set(cl.rsv_arr["node"].tolist())
    assert any(n in rnodes for n in nodes.tolist())   # some pods land on reservation nodes
