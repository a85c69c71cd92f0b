"""Named scalar slots (kg_config.ext_resource_names, KG_RES_EXT0..4): the extended resources and hugepages a
deployment's pods request — nvidia.com/gpu, koordinator.sh/gpu-core, koordinator.sh/rdma, hugepages-2Mi, several at
once — instead of one slot hard-wired to example.com/gpu.  Upstream NodeResourcesFit's fitsRequest compares every
requested scalar resource (the in-repo mirror: reservation/plugin.go:469-473), its scorer weighs the ones the
ScoringStrategy names, LoadAware weighs the ones resourceWeights name.  Checked on the host: config validation,
the ingest's name map, the sorted-name order the topology merge walks, and the per-pair code (kg_row_eval) and
Reserve (kg_row_commit) against the oracle on clusters requesting up to three of them at once.  (The reference's
tests weigh cpu / memory only: beyond them this is parity against the oracle's restatement.)"""
import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, ingest, objects, synth
from koordinator_amd.config import make_config, shipped_profile
from oracle import oracle

NAMES = synth.SCALAR_NAMES


def _validate(cfg):
    import ctypes
    err = ctypes.create_string_buffer(256)
    st = nat.lib().kg_config_validate(nat.ptr(cfg), err, 256)
    return st, err.value.decode()


def test_config_names_default_and_validation():
    cfg = make_config()
    assert cfg["ext_resource_names"][0] == b"example.com/gpu" and cfg["ext_resource_names"][1] == b""
    assert _validate(cfg)[0] == 0
    cfg = make_config(extended_resources=NAMES)
    assert [n.decode() for n in cfg["ext_resource_names"][:4]] == list(NAMES)
    assert _validate(cfg)[0] == 0
    bad = cfg.copy()
    bad["ext_resource_names"][1] = b"nvidia.com/gpu"
    st, msg = _validate(bad)
    assert st != 0 and "repeats" in msg
    bad = cfg.copy()
    bad["ext_resource_names"][2] = b"memory"
    assert _validate(bad)[0] != 0
    with pytest.raises(ValueError):
        objects.resource_map(("a", "b", "c", "d", "e", "f"))


def test_ingest_maps_names_to_slots():
    pod = {"metadata": {"name": "p", "namespace": "d"},
           "spec": {"containers": [{"resources": {"requests": {"cpu": "1", "nvidia.com/gpu": "2",
                                                               "koordinator.sh/rdma": "1", "hugepages-2Mi": "64Mi"}}}]}}
    with pytest.raises(ingest.UnsupportedResource):
        ingest.pod_from_object(pod)
    with objects.extended_resources(NAMES):
        p = ingest.pod_from_object(pod)
        rl = objects.resource_list(p.containers[0].requests)
        assert rl["v"][nat.RES_EXT0] == 2 and rl["v"][nat.RES_EXT2] == 1 and rl["v"][nat.RES_EXT3] == 64 << 20
        assert rl["present"] == (1 << nat.RES_CPU) | (1 << nat.RES_EXT0) | (1 << nat.RES_EXT2) | (1 << nat.RES_EXT3)
    assert objects.RES.get("nvidia.com/gpu") is None   # restored to the default names


def _pairs(cfg, cl, P, N):
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    out = np.zeros((3, P, N), np.int64)
    for i in range(P):
        for j in range(N):
            out[:, i, j] = engine.row_eval(cfg, nodes[j:j + 1], pods[i:i + 1], cl.now_ns)[:3]
    return out


PROFILES = {
    "fit_gpu_rdma": dict(fit_resources={"cpu": 1, "memory": 1, "nvidia.com/gpu": 2, "koordinator.sh/rdma": 1}),
    "most_all": dict(fit_strategy="MostAllocated",
                     fit_resources={"cpu": 1, "memory": 1, "nvidia.com/gpu": 1, "koordinator.sh/gpu-core": 1,
                                    "koordinator.sh/rdma": 1, "hugepages-2Mi": 1}),
    "la_gpu_core": dict(resource_weights={"cpu": 1, "memory": 1, "koordinator.sh/gpu-core": 2},
                        estimated_scaling_factors={"koordinator.sh/gpu-core": 100}),
}


@pytest.mark.parametrize("name", sorted(PROFILES))
def test_row_eval_named_scalars_match_oracle(name):
    P, N = 48, 160
    cl = synth.make_scalar_cluster(N, P, seed=61)
    cfg = shipped_profile(extended_resources=NAMES, **PROFILES[name])
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    assert ((pods["request_present"] >> nat.RES_EXT0) & 0xF != 0).sum() > P // 5   # pods request the named slots
    assert (np.array([bin(int(x) >> nat.RES_EXT0 & 0xF).count("1") for x in pods["request_present"]]) >= 2).any()
    got = _pairs(cfg, cl, P, N)
    m, f, l = oracle.eval_matrix(cfg, cl, np.arange(P), cl.now_ns)
    np.testing.assert_array_equal(got[0].astype(bool), m)
    np.testing.assert_array_equal(got[1], f)
    np.testing.assert_array_equal(got[2], l)
    # the named slots decide feasibility: dropping their requests frees pods somewhere
    cl2 = synth.make_scalar_cluster(N, P, seed=61)
    cl2.containers["requests"]["present"] &= np.uint32(~(0xF << nat.RES_EXT0) & 0xFFFFFFFF)
    m2 = oracle.eval_matrix(cfg, cl2, np.arange(P), cl.now_ns)[0]
    assert (m2 & ~m).any()


def test_schedule_named_scalars_commit_matches_oracle():
    """The sequential cycle with Reserve adding the named slots' requests (kg_row_commit), pods with two or three
    scalar requests landing on the same nodes until one of them runs out."""
    P, N = 120, 40
    cl = synth.make_scalar_cluster(N, P, seed=62)
    cfg = shipped_profile(extended_resources=NAMES, **PROFILES["fit_gpu_rdma"])
    ref_n, ref_s = oracle.schedule(cfg, cl, np.arange(P), cl.now_ns)
    nodes = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, np.arange(P))
    for p in range(P):
        best, bn = -1, -1
        for j in range(N):
            ok, fs, ls = engine.row_eval(cfg, nodes[j:j + 1], pods[p:p + 1], cl.now_ns)[:3]
            if ok:
                t = fs * cfg["weight_fit"] + ls * cfg["weight_loadaware"]
                if t > best:
                    best, bn = t, j
        assert bn == ref_n[p], p
        if bn >= 0:
            assert best == ref_s[p]
            engine.row_commit(cfg, nodes[bn:bn + 1], pods[p:p + 1])
    assert (ref_n == -1).any() and (ref_n >= 0).sum() > P // 2


def test_sorted_name_order_follows_names():
    """The topology merge walks the hint lists in sorted resource-name order (Go string order): a named slot sorting
    before "cpu" moves ahead of it, unused slots go last.  The oracle's order against Python's sort of the names."""
    ext = ("a.example/first", "", "zz.example/last", "hugepages-1Gi")
    cfg = make_config(extended_resources=ext)
    rmap = objects.resource_map(ext)
    want = [r for _, r in sorted(rmap.items())] + [r for r in range(nat.NUM_RES) if r not in rmap.values()]
    assert oracle.sorted_res_order(cfg).tolist() == want
    assert want[0] == nat.RES_EXT0 and want[-1] == nat.RES_EXT4
