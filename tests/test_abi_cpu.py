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
from rows_ref import rows_eval

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


def test_header_constants_match_python():
    import re
    text = open(HEADER).read()
    consts = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define (KG_\w+) (\d+)\b", text)}
    assert consts["KG_ABI_VERSION"] == nat.ABI_VERSION
    assert consts["KG_PLACE_CHUNK_MAX"] == nat.PLACE_CHUNK_MAX
    assert consts["KG_PARTIAL_SLOTS"] == nat.PARTIAL_SLOTS


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
    extra = good.copy()
    extra["la_resource_weight"][3] = 1  # LoadAware weights beyond cpu/memory: the exact pair path
    assert L.kg_config_validate(nat.ptr(extra), buf, 256) == 0
    for chunk, ok in ((-1, False), (0, True), (1, True), (1024, True), (1025, False)):
        c = good.copy()
        c["place_chunk"] = chunk        # kg_place: 0 ⇒ default 16, at most KG_PLACE_CHUNK_MAX
        assert (L.kg_config_validate(nat.ptr(c), buf, 256) == 0) == ok, chunk


def test_place_chunk_rule_matches_kg_place():
    from koordinator_amd import dist as kdist
    cfg = shipped_profile()
    for chunk, want in ((0, 16), (1, 1), (64, 64), (1024, 1024), (5000, 1024)):
        cfg["place_chunk"] = chunk
        assert kdist.place_chunk_of(cfg) == want
    cfg["place_chunk"] = -3
    with pytest.raises(ValueError):
        kdist.place_chunk_of(cfg)
    with pytest.raises(ValueError):
        kdist.place_sharded(None, 0, None, chunk=0)


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
