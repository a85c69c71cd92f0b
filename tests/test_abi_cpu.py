"""CPU-only checks of the boundary and the host logic (no GPU calls).

* the engine library loads and exports every function ``include/koord_gpu.h`` declares, with the
  struct layouts the Python mirror assumes;
* the host row builders (``kg_build_pod_rows`` / ``kg_build_node_rows`` / ``kg_row_commit``) carry
  everything the kernels need: an exact int64 evaluation written over the rows alone (the pair
  formulas the kernels implement) reproduces the oracle's object-level Filter/Score matrices.
"""
import os
import re

import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle

HEADER = os.path.join(os.path.dirname(__file__), "..", "include", "koord_gpu.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(kg_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if not n.startswith("kg_mask_test")))


def test_library_exports_every_declared_function():
    L = nat.lib()
    decl = declared_functions()
    assert len(decl) >= 25
    missing = [n for n in decl if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(decl) == sorted(nat.EXPORTED)


def test_struct_layouts_match():
    nat.check_abi()
    assert nat.lib().kg_abi_version() == nat.ABI_VERSION


def test_config_validation_rejects_bad_args():
    import ctypes
    L = nat.lib()
    buf = ctypes.create_string_buffer(256)
    good = shipped_profile()
    assert L.kg_config_validate(nat.ptr(good), buf, 256) == 0
    bad = good.copy()
    bad["weight_fit"] = 30000
    bad["weight_loadaware"] = 30000     # totals would overflow the 32-bit tile keys
    assert L.kg_config_validate(nat.ptr(bad), buf, 256) != 0
    bad = good.copy()
    bad["la_resource_weight"][3] = 1    # LoadAware weights beyond cpu/memory are unsupported
    assert L.kg_config_validate(nat.ptr(bad), buf, 256) != 0


def _lr(req, cap):
    """LR(req, cap) = req > cap ? 0 : (cap - req) * 100 / cap, int64 (cap > 0)."""
    safe = np.where(cap > 0, cap, 1)
    q = ((safe - req) * 100) // safe
    return np.where((cap > 0) & (req <= cap), q, 0)


def _mr(req, cap):
    safe = np.where(cap > 0, cap, 1)
    return np.where(cap > 0, (np.minimum(req, safe) * 100) // safe, 0)


def rows_eval(cfg, nodes, pods, now_ns):
    """Exact evaluation of every (pod, node) pair from engine rows only (mirrors kg_pair_exact)."""
    N, P = len(nodes), len(pods)
    fit_on = bool(cfg["enabled_plugins"] & nat.PLUGIN_FIT)
    la_on = bool(cfg["enabled_plugins"] & nat.PLUGIN_LOADAWARE)
    most = int(cfg["fit_strategy"]) == nat.STRATEGY_MOST_ALLOCATED
    fw = cfg["fit_resource_weight"].astype(np.int64)
    lw = cfg["la_resource_weight"].astype(np.int64)
    valid = (nodes["flags"] & nat.NODE_VALID) != 0
    full = nodes["pod_count"].astype(np.int64) + 1 > nodes["allowed_pods"].astype(np.int64)
    has_metric = (nodes["flags"] & nat.NODE_HAS_METRIC) != 0
    has_upd = (nodes["flags"] & nat.NODE_HAS_UPDATE_TIME) != 0
    exp_ns = int(cfg["la_expiration_seconds"]) * 10**9 if cfg["la_has_expiration"] else 0
    expired = ~has_upd | ((exp_ns > 0) & (now_ns - nodes["metric_update_ns"] >= exp_ns))
    skip_filter = bool(cfg["la_filter_expired_node_metrics"]) and bool(cfg["la_has_expiration"])
    la_valid = has_metric & ~(bool(cfg["la_has_expiration"]) & expired)
    free = nodes["alloc"] - nodes["requested"]
    mask = np.zeros((P, N), bool)
    fit = np.zeros((P, N), np.int64)
    la = np.zeros((P, N), np.int64)
    for i, p in enumerate(pods):
        ok = valid.copy()
        if fit_on:
            ok &= ~full
            if p["flags"] & nat.POD_HAS_REQUEST:
                for r in range(nat.NUM_RES):
                    if r < 3 or (p["request_present"] >> r) & 1:
                        ok &= p["request"][r] <= free[:, r]
        if la_on and not (p["flags"] & nat.POD_DAEMONSET):
            bit = nat.NODE_LA_PASS_PROD if p["flags"] & nat.POD_PROD else nat.NODE_LA_PASS_NONPROD
            passes = ~has_metric | (skip_filter & expired) | ((nodes["flags"] & bit) != 0)
            ok &= passes
        mask[i] = ok
        if fit_on:
            s = np.zeros(N, np.int64)
            w = np.zeros(N, np.int64)
            for r in range(nat.NUM_RES):
                pr = int(p["fit_score_request"][r])
                if fw[r] <= 0 or (r >= 3 and pr == 0):
                    continue
                a = nodes["alloc"][:, r]
                present = np.ones(N, bool) if r < 3 else ((nodes["alloc_present"] >> r) & 1) == 1
                use = present & (a != 0)
                base = nodes["nonzero_requested"][:, r] if r < 2 else nodes["requested"][:, r]
                q = _mr(base + pr, a) if most else _lr(base + pr, a)
                s += np.where(use, q * fw[r], 0)
                w += np.where(use, fw[r], 0)
            fit[i] = np.where(w > 0, s // np.where(w > 0, w, 1), 0)
        if la_on:
            v = 1 if p["flags"] & nat.POD_LA_PROD_SCORE else 0
            s = np.zeros(N, np.int64)
            for r in range(2):
                if lw[r] == 0:
                    continue
                s += _lr(p["la_estimate"][r] + nodes["la_used"][:, v, r], nodes["la_alloc"][:, r]) * lw[r]
            la[i] = np.where(la_valid, s // max(int(lw[:2].sum()), 1), 0)
    return mask, fit, la


@pytest.mark.parametrize("profile", ["default", "shipped", "most"])
def test_rows_carry_the_oracle_semantics(profile):
    cl = synth.make_cluster(3_000, 120, seed=41)
    cfg = {"default": make_config, "shipped": shipped_profile,
           "most": lambda: make_config(fit_strategy="MostAllocated",
                                       fit_resources={"cpu": 2, "memory": 1, "kubernetes.io/batch-memory": 3})}[profile]()
    idx = np.arange(120)
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    m, f, l = rows_eval(cfg, nodes, pods, cl.now_ns)
    m_ref, f_ref, l_ref = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(m, m_ref)
    np.testing.assert_array_equal(f, f_ref)
    np.testing.assert_array_equal(l, l_ref)


def test_row_commit_matches_sequential_oracle():
    """Sequential placement over rows (exact eval + kg_row_commit) == the oracle's cycle."""
    cl = synth.make_cluster(400, 150, seed=43)
    cfg = shipped_profile()
    idx = np.arange(150)
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    got_n, got_s = [], []
    for i in range(len(pods)):
        m, f, l = rows_eval(cfg, nodes, pods[i:i + 1], cl.now_ns)
        tot = np.where(m[0], int(cfg["weight_fit"]) * f[0] + int(cfg["weight_loadaware"]) * l[0], -1)
        j = int(tot.argmax())
        if tot[j] < 0:
            got_n.append(-1)
            got_s.append(-1)
            continue
        got_n.append(j)
        got_s.append(int(tot[j]))
        engine.row_commit(cfg, nodes[j:j + 1], pods[i:i + 1])
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(np.array(got_n), ref_n)
    np.testing.assert_array_equal(np.array(got_s), ref_s)
