"""Reservation / ElasticQuota on the CPU: the oracle and the engine's shared per-pair code
(kg_row_eval_rsv) against the reference's TestScore known answers, and the host-row mirror of the
engine's per-pod reduction against the oracle on seeded config-5 clusters."""
import numpy as np
import pytest

from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle
from rsv_cases import kat_cluster, kat_doc, rows_matrix5, rsv_cluster

DOC = kat_doc()
RSV = ("NodeResourcesFit", "LoadAwareScheduling", "Reservation")


@pytest.mark.parametrize("case", DOC["cases"], ids=lambda c: c["name"])
def test_reservation_score_kat(case):
    cfg = make_config(plugins=("Reservation",))
    view = kat_cluster(DOC, case)
    ok, raw, nom = oracle.rsv_pair(cfg, view, 0, 0)
    assert raw == case["want"]
    rows = engine.build_node_rows(cfg, view)
    prow = engine.build_pod_rows(cfg, view, [0])
    f, _, _, _, raw2, _, nom2 = engine.row_eval_rsv(cfg, rows[0:1], view.rsv_arr, prow[0:1], view.now_ns)
    assert (f, raw2, nom2) == (ok, raw, nom)


@pytest.mark.parametrize("seed", [51, 52])
def test_rows_match_oracle_matrix(seed):
    cl = rsv_cluster(600, 24, seed=seed, rsv_node_frac=0.3)
    cfg = shipped_profile(plugins=RSV)
    idx = np.arange(24)
    got = rows_matrix5(cfg, cl, idx, cl.now_ns)
    m, fit, la, numa, rsv, top1 = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    for a, b in zip(got, (m, fit, la, numa, rsv, top1)):
        np.testing.assert_array_equal(a, b)
    assert rsv.max() == 100 and m.any()


def test_rows_match_oracle_many_reservations_per_node():
    """Up to KG_MAX_RSV_PER_NODE (16) reservations on a node (the reservation cache is unbounded,
    cache.go:60,252)."""
    cl = rsv_cluster(300, 24, seed=77, rsv_node_frac=0.3, max_rsv_per_node=16)
    counts = np.bincount(cl.rsv_arr["node"])
    assert counts.max() > 8
    cfg = shipped_profile(plugins=RSV)
    idx = np.arange(24)
    got = rows_matrix5(cfg, cl, idx, cl.now_ns)
    want = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("seed", [54, 55])
def test_rows_match_oracle_matrix_with_numa(seed):
    """Reservation + NodeNUMAResource (the shipped profile's filter set without ElasticQuota): the
    NUMA terms of reservation nodes run on the restored NodeInfo (kg_rsv_pair → kg_numa_pair)."""
    cl = synth.make_profile_cluster(400, 24, seed=seed, rsv_node_frac=0.4)
    cfg = shipped_profile(plugins=RSV + ("NodeNUMAResource",), weight_numa=2)
    idx = np.arange(24)
    got = rows_matrix5(cfg, cl, idx, cl.now_ns)
    m, fit, la, numa, rsv, top1 = oracle.eval_matrix5(cfg, cl, idx, cl.now_ns)
    for a, b in zip(got, (m, fit, la, numa, rsv, top1)):
        np.testing.assert_array_equal(a, b)
    assert rsv.max() == 100 and m.any() and numa.any()


def test_oracle_quota_gate_and_reserve():
    """ElasticQuota: pods beyond the group's runtime are unschedulable; used grows by the placed
    pods' requests (oracle invariants on a config-5 cluster)."""
    cl = rsv_cluster(400, 300, seed=53, n_quotas=4, quota_ratio=0.3)
    cfg = shipped_profile(plugins=RSV + ("ElasticQuota",))
    nodes, scores, rsv, quota = oracle.schedule2(cfg, cl, np.arange(300), cl.now_ns)
    assert (nodes == -1).any() and (nodes >= 0).any()
    req = cl.containers["requests"]["v"]
    for g in range(4):
        placed = (nodes >= 0) & (cl.pods["quota"] == g)
        for r in (3, 4):
            assert quota["used"]["v"][g, r] == req[placed, r].sum()
            assert quota["used"]["v"][g, r] <= cl.quota_arr["used_limit"]["v"][g, r]
    # every placement on a node with a nominated reservation added to that reservation
    assert (rsv["n_assigned"] >= cl.rsv_arr["n_assigned"]).all()


@pytest.mark.parametrize("check_parent", [0, 1])
def test_oracle_quota_tree_reserve_and_parent_gate(check_parent):
    """ElasticQuota over a quota tree: Reserve adds the pod's requests to its group and every ancestor
    (updateGroupDeltaUsedNoLock); with EnableCheckParentQuota every ancestor's used stays within its
    limit, without it only the pod's own group's does."""
    cl = rsv_cluster(400, 300, seed=54, n_quotas=7, quota_ratio=0.5, quota_tree=True)
    assert list(cl.quota_arr["parent"]) == [-1, 0, 0, 1, 1, 2, 2]
    cfg = shipped_profile(plugins=RSV + ("ElasticQuota",), eq_check_parent_quota=check_parent)
    nodes, _, _, quota = oracle.schedule2(cfg, cl, np.arange(300), cl.now_ns)
    req = cl.containers["requests"]["v"]
    sub = {g: {g} for g in range(7)}
    for g in range(6, 0, -1):
        sub[(g - 1) // 2] |= sub[g]
    over = False
    for g in range(7):
        placed = (nodes >= 0) & np.isin(cl.pods["quota"], sorted(sub[g]))
        own = (nodes >= 0) & (cl.pods["quota"] == g)
        for r in (3, 4):
            assert quota["used"]["v"][g, r] == req[placed, r].sum()
            assert req[own, r].sum() <= cl.quota_arr["used_limit"]["v"][g, r]
            over |= quota["used"]["v"][g, r] > cl.quota_arr["used_limit"]["v"][g, r]
    assert over == (not check_parent)
