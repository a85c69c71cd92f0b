"""Named scalar slots on the GPU (kg_config.ext_resource_names): pods requesting up to three of nvidia.com/gpu,
koordinator.sh/gpu-core, koordinator.sh/rdma, hugepages-2Mi at once, through every engine path — matrix mode (the
class kernels and the slot kernel with the batch's 8-slot resource map, full planes against the oracle), placement
(kg_place: touched-node re-scores and Reserve on the named slots, against the oracle's cycle and the host replay),
LoadAware weights on a named slot (the LAX form), and the NodeNUMAResource + Reservation + ElasticQuota profile."""
import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu

NAMES = synth.SCALAR_NAMES
PROFILES = {
    "fit_gpu_rdma": dict(fit_resources={"cpu": 1, "memory": 1, "kubernetes.io/batch-cpu": 1,
                                        "kubernetes.io/batch-memory": 1, "nvidia.com/gpu": 2, "koordinator.sh/rdma": 1}),
    "most_all": dict(fit_strategy="MostAllocated",
                     fit_resources={"cpu": 1, "memory": 1, "nvidia.com/gpu": 1, "koordinator.sh/gpu-core": 1,
                                    "koordinator.sh/rdma": 1, "hugepages-2Mi": 1}),
    "la_gpu_core": dict(resource_weights={"cpu": 1, "memory": 1, "koordinator.sh/gpu-core": 2},
                        estimated_scaling_factors={"koordinator.sh/gpu-core": 100}),
}


def _replay(cfg, cl, idx, nodes):
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes.tolist()):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    return rows


@pytest.mark.parametrize("name", sorted(PROFILES))
def test_matrix_named_scalars(name):
    P, N = 300, 3_000
    cl = synth.make_scalar_cluster(N, P, seed=71)
    cfg = shipped_profile(extended_resources=NAMES, **PROFILES[name])
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        out = eng.eval(cl.now_ns)
    m, f, l = oracle.eval_matrix(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(engine.unpack_mask(out["mask"], N), m)
    np.testing.assert_array_equal(out["scores"][:, :N, 0], np.where(m, f, out["scores"][:, :N, 0]))
    np.testing.assert_array_equal(out["scores"][:, :N, 1], np.where(m, l, out["scores"][:, :N, 1]))
    t = np.where(m, f.astype(np.int64) + l, -1)
    node, tot = engine.decode_top1(out["top1"])
    np.testing.assert_array_equal(node, np.where(t.max(axis=1) >= 0, t.argmax(axis=1), -1))


@pytest.mark.parametrize("name", ["fit_gpu_rdma", "most_all"])
def test_place_named_scalars(name):
    P, N = 400, 1_100
    cl = synth.make_scalar_cluster(N, P, seed=72)
    cfg = shipped_profile(extended_resources=NAMES, place_chunk=16, **PROFILES[name])
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))
    assert (after["requested"][:, nat.RES_EXT0:nat.RES_EXT3 + 1] > engine.build_node_rows(cfg, cl)["requested"][
        :, nat.RES_EXT0:nat.RES_EXT3 + 1]).any()


def test_shipped_profile_numa_rsv_quota_named_scalars():
    """The whole shipped profile (NodeNUMAResource, Reservation, ElasticQuota) on a cluster whose pods request the
    named slots: reservations and quotas carry them too (quotav1 sums over every key)."""
    from rsv_cases import rsv_cluster
    P, N = 200, 2_000
    cl = rsv_cluster(N, P, seed=73, n_quotas=6, quota_ratio=0.7)
    sc = synth.make_scalar_cluster(N, P, seed=73)
    cl.containers["requests"]["v"][:, nat.RES_EXT0:] = sc.containers["requests"]["v"][:len(cl.containers), nat.RES_EXT0:]
    cl.containers["requests"]["present"] |= sc.containers["requests"]["present"][:len(cl.containers)] & np.uint32(0xF80)
    cl.nodes["allocatable"]["v"][:, nat.RES_EXT0:] = sc.nodes["allocatable"]["v"][:, nat.RES_EXT0:]
    cl.nodes["allocatable"]["present"] |= sc.nodes["allocatable"]["present"] & np.uint32(0xF80)
    cfg = shipped_profile(extended_resources=NAMES, plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation",
                                                             "ElasticQuota"), **PROFILES["fit_gpu_rdma"])
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        q_after = eng.download_quotas()
    ref_n, ref_s, _, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
