"""kg_place's pipeline (chunk i + 1 evaluated while chunk i commits; its resolve re-scores chunk i's nodes)
forced on and off, on clusters small enough that consecutive chunks keep choosing the same nodes — the case
where a stale key of a node chunk i committed could win if the re-score were missing.  Both NodeNUMAResource
chunk forms (k_eval_numa_chunk's top-16 lists and k_eval_numa2's one key per tile, KG_FORM_NUMA_CHUNK_TILE) and
the Fit + LoadAware chunk kernel; placements and scores against the oracle's sequential cycle, node rows
against the host replay."""
import numpy as np
import pytest

from koordinator_amd import _native as nat
from koordinator_amd import engine, synth
from koordinator_amd.config import shipped_profile
from oracle import oracle

pytestmark = pytest.mark.gpu


def _replay(cfg, cl, idx, nodes):
    rows = engine.build_node_rows(cfg, cl)
    prow = engine.build_pod_rows(cfg, cl, idx)
    for p, n in enumerate(nodes.tolist()):
        if n >= 0:
            engine.row_commit(cfg, rows[n:n + 1], prow[p:p + 1])
    return rows


@pytest.mark.parametrize("chunk_form", ["topk", "topk_nocache", "tile_key"])
@pytest.mark.parametrize("pipeline", ["1", "0"])
@pytest.mark.parametrize("n_nodes", [1024, 2000])
def test_numa_place_pipeline_on_off(n_nodes, pipeline, chunk_form):
    """The pipelined "topk" form of a batch of repeated pod rows (~50 distinct of 240) reads the distinct rows'
    cached NodeNUMAResource outcomes (k_eval_numa_cached, refreshed per chunk); "topk_nocache" evaluates every pair."""
    forms = (0 if pipeline == "1" else nat.FORM_PLACE_SEQUENTIAL) | (nat.FORM_NUMA_CHUNK_TILE if chunk_form == "tile_key" else 0)
    forms |= nat.FORM_NUMA_NO_CACHE if chunk_form == "topk_nocache" else 0
    P = 240
    cl = synth.make_numa_cluster(n_nodes, P, seed=91 + n_nodes)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.set_forms(forms)
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    if chunk_form == "topk":   # the cache's precondition: the batch repeats rows (pod equivalence on)
        rows = engine.build_pod_rows(cfg, cl, idx)
        assert 4 * len({r.tobytes() for r in rows}) <= 3 * P
    # consecutive chunks (16 pods) land on common nodes: the re-score of the previous chunk's nodes matters
    placed = nodes[nodes >= 0]
    chunks = [set(placed[i:i + 16].tolist()) for i in range(0, len(placed), 16)]
    assert sum(len(a & b) > 0 for a, b in zip(chunks, chunks[1:])) > 3
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))


@pytest.mark.parametrize("pipeline", ["2", "0"])
def test_fit_loadaware_place_pipeline_on_off(pipeline):
    """The Fit + LoadAware batch takes the sequential form by default; forced on (KG_FORM_PLACE_PIPELINE), the
    pipeline must agree."""
    P = 600
    cl = synth.make_cluster(1024, P, seed=93)
    cfg = shipped_profile()
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.set_forms(nat.FORM_PLACE_PIPELINE if pipeline == "2" else 0)
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)


@pytest.mark.parametrize("kind", ["fit_la", "fit_la_pipe_most", "numa", "quota"])
def test_resolve_small_clusters(kind):
    """k_resolve against the oracle's cycle on small clusters, so pods keep landing on nodes the previous pod
    took (the touched-node re-score right after a Reserve); an ElasticQuota tree without Reservation (the gate
    after each Reserve).  "fit_la_pipe_most": the plain form pipelined (KG_FORM_PLACE_PIPELINE) under MostAllocated,
    so a node the previous chunk committed is committed again by an earlier pod of the chunk and then scored by a
    later one (the previous-chunk loop must leave it to the touched re-score: its global row may still be in flight
    behind the plain form's LDS-only barriers)."""
    from rsv_cases import rsv_cluster
    P = 300
    if kind == "fit_la":
        cl = synth.make_cluster(1024, P, seed=95)
        cfg = shipped_profile(place_chunk=16)
    elif kind == "fit_la_pipe_most":
        cl = synth.make_cluster(1024, P, seed=98)
        cfg = shipped_profile(place_chunk=16, fit_strategy="MostAllocated")
    elif kind == "numa":
        cl = synth.make_numa_cluster(1500, P, seed=96)
        cfg = shipped_profile()
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    else:
        cl = rsv_cluster(2000, P, seed=97, n_quotas=15, quota_ratio=0.5, quota_tree=True)
        cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "ElasticQuota"),
                              eq_check_parent_quota=1)
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        if kind == "fit_la_pipe_most":
            eng.set_forms(nat.FORM_PLACE_PIPELINE)
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        if kind == "quota":
            eng.set_quotas(cl.quota_arr)
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
        q_after = eng.download_quotas() if kind == "quota" else None
    if kind == "quota":
        ref_n, ref_s, _, ref_q = oracle.schedule2(cfg, cl, idx, cl.now_ns)
        assert (ref_n == -1).any() and (ref_n >= 0).any()
        np.testing.assert_array_equal(q_after["used"]["v"], ref_q["used"]["v"])
    else:
        ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    if kind == "fit_la":
        assert (np.diff(nodes[nodes >= 0]) == 0).any()   # back-to-back pods on one node
    if kind == "fit_la_pipe_most":
        # the shape the previous-chunk loop must handle: a node of chunk i − 1 committed twice in chunk i
        hits = 0
        for b in range(16, P, 16):
            prev, cur = set(nodes[b - 16:b].tolist()) - {-1}, nodes[b:b + 16].tolist()
            hits += sum(1 for n in set(cur) if n in prev and cur.count(n) >= 2)
        assert hits > 3, hits
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))
