"""kg_place's pipeline (chunk i + 1 evaluated while chunk i commits; its resolve re-scores chunk i's nodes)
forced on and off, on clusters small enough that consecutive chunks keep choosing the same nodes — the case
where a stale key of a node chunk i committed could win if the re-score were missing.  Both NodeNUMAResource
chunk forms (k_eval_numa_chunk's top-16 lists and k_eval_numa2's one key per tile, KG_NUMA_CHUNK_PODS=0) and
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


@pytest.mark.parametrize("chunk_form", ["topk", "tile_key"])
@pytest.mark.parametrize("pipeline", ["1", "0"])
@pytest.mark.parametrize("n_nodes", [1024, 2000])
def test_numa_place_pipeline_on_off(n_nodes, pipeline, chunk_form, monkeypatch):
    monkeypatch.setenv("KG_PLACE_PIPELINE", pipeline)
    if chunk_form == "tile_key":
        monkeypatch.setenv("KG_NUMA_CHUNK_PODS", "0")
    P = 240
    cl = synth.make_numa_cluster(n_nodes, P, seed=91 + n_nodes)
    cfg = shipped_profile()
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
        after = eng.download()
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    # consecutive chunks (16 pods) land on common nodes: the re-score of the previous chunk's nodes matters
    placed = nodes[nodes >= 0]
    chunks = [set(placed[i:i + 16].tolist()) for i in range(0, len(placed), 16)]
    assert sum(len(a & b) > 0 for a, b in zip(chunks, chunks[1:])) > 3
    np.testing.assert_array_equal(after, _replay(cfg, cl, idx, nodes))


@pytest.mark.parametrize("pipeline", ["2", "0"])
def test_fit_loadaware_place_pipeline_on_off(pipeline, monkeypatch):
    """The Fit + LoadAware batch takes the sequential form by default; forced on (KG_PLACE_PIPELINE=2), the
    pipeline must agree."""
    monkeypatch.setenv("KG_PLACE_PIPELINE", pipeline)
    P = 600
    cl = synth.make_cluster(1024, P, seed=93)
    cfg = shipped_profile()
    idx = np.arange(P)
    with engine.Engine(cfg) as eng:
        eng.load_snapshot(engine.build_node_rows(cfg, cl))
        eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
        nodes, scores = eng.place(cl.now_ns)
    ref_n, ref_s = oracle.schedule(cfg, cl, idx, cl.now_ns)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
