"""The shape of round 5's unexplained illegal address (`test_numa_place_pipeline_on_off
[1024-1-topk]`, the pipelined NodeNUMAResource placement with the outcome cache on 1,024 nodes), made harder: a short
last chunk, unschedulable pods interleaved so the previous-chunk lists carry −1, every pipelined form (outcome cache
on and off, one key per tile, the plain Fit + LoadAware pipeline), and a two-rank sharded run whose second shard starts
above node 0 (the cache's column offset).  Each runs twice: on the product library against the oracle's cycle, and on
the bounds-checked build (libkoordgpu_bounds.so, -DKG_BOUNDS_CHECK: every index into the previous-chunk lists,
pvkeys, the outcome cache, the touched / rescan lists and the slow list is checked on the device, a violation is
reported by kg_place instead of being performed), which must report none and place identically."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_SO = os.path.join(ROOT, "koordinator_amd", "lib", "libkoordgpu_bounds.so")
P = 16 * 17 + 5   # 17 full chunks of 16 and a short last one


def _case(form):
    from koordinator_amd import _native as nat
    from koordinator_amd import engine, synth
    from koordinator_amd.config import shipped_profile
    if form == "plain_pipe":
        cl = synth.make_cluster(1_024, P, seed=101)
        cfg = shipped_profile(place_chunk=16, fit_strategy="MostAllocated")
        forms = nat.FORM_PLACE_PIPELINE
    else:
        # (the two-rank form needs a second shard: 2,048 nodes, shards [0, 1024) and [1024, 2048))
        cl = synth.make_numa_cluster(2_048 if form == "sharded_cache" else 1_024, P, seed=91 + 1_024)
        cfg = shipped_profile()
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
        forms = {"cache": 0, "nocache": nat.FORM_NUMA_NO_CACHE, "tile": nat.FORM_NUMA_CHUNK_TILE,
                 "sharded_cache": 0}[form]
    idx = np.arange(P)
    # unschedulable pods: a cpu (or batch-cpu) request of 10^6 cores, every 7th pod — their chunk's previous-chunk list
    # then carries −1 (the cluster is edited in place: its C view points at these arrays)
    bad = idx[idx % 7 == 3]
    rq = cl.containers["requests"]
    for r in (nat.RES_CPU, nat.RES_BATCH_CPU):
        has = (rq["present"][bad] >> r) & 1 == 1
        rq["v"][bad[has], r] = 10**9
    rows = engine.build_node_rows(cfg, cl)
    pods = engine.build_pod_rows(cfg, cl, idx)
    return cl, cfg, rows, pods, idx, forms, bad


def _oracle(form):
    from oracle import oracle
    cl, cfg, rows, pods, idx, forms, bad = _case(form)
    return oracle.schedule(cfg, cl, idx, cl.now_ns)


def _place(form):
    """Runs in this process (product library) or in a child with KG_ENGINE_SO set (bounds build)."""
    from koordinator_amd import engine
    cl, cfg, rows, pods, idx, forms, bad = _case(form)
    with engine.Engine(cfg) as eng:
        eng.set_forms(forms)
        eng.load_snapshot(rows)
        eng.set_pods(pods)
        nodes, scores = eng.place(cl.now_ns)
    return nodes, scores


def _sharded(form, so, world=2):
    """Two ranks on one GPU (loopback communicator), every rank on `so`."""
    code = ("import sys, json, numpy as np; sys.path[:0] = [%r, %r]\n"
            "import test_bounds_gpu as t\n"
            "from koordinator_amd import dist as kdist\n"
            "import torch\n"
            "rank, world, name = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]\n"
            "cl, cfg, rows, pods, idx, forms, bad = t._case(%r)\n"
            "eng = kdist.native_engine(cfg, rows, pods, torch.device('cuda', 0), comm='loopback', rank=rank, world=world, shm_name=name)\n"
            "eng.set_forms(forms)\n"
            "n, s = eng.place_sharded(cl.now_ns)\n"
            "eng.close()\n"
            "print('RESULT ' + json.dumps([n.tolist(), s.tolist()]))\n") % (ROOT, os.path.dirname(__file__), form)
    env = dict(os.environ)
    if so:
        env["KG_ENGINE_SO"] = so
    name = f"/kg_bounds_{os.getpid()}"
    ps = [subprocess.Popen([sys.executable, "-c", code, str(r), str(world), name], env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True) for r in range(world)]
    outs = []
    for p in ps:
        o, e = p.communicate(timeout=180)
        assert p.returncode == 0, e[-3000:]
        line = [ln for ln in o.splitlines() if ln.startswith("RESULT ")][-1]
        outs.append(json.loads(line[len("RESULT "):]))
    return outs


def _child_place(form, so):
    code = ("import sys, json; sys.path[:0] = [%r, %r]\n"
            "import test_bounds_gpu as t\n"
            "n, s = t._place(%r)\n"
            "print('RESULT ' + json.dumps([n.tolist(), s.tolist()]))\n") % (ROOT, os.path.dirname(__file__), form)
    r = subprocess.run([sys.executable, "-c", code], env={**os.environ, "KG_ENGINE_SO": so}, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    n, s = json.loads(line[len("RESULT "):])
    return np.asarray(n, np.int32), np.asarray(s, np.int64)


@pytest.mark.parametrize("form", ["cache", "nocache", "tile", "plain_pipe"])
def test_pipeline_short_last_chunk_unplaced(form):
    ref_n, ref_s = _oracle(form)
    cl, cfg, rows, pods, idx, forms, bad = _case(form)
    assert (ref_n[bad] == -1).all() and (ref_n >= 0).sum() > P // 2
    nodes, scores = _place(form)
    np.testing.assert_array_equal(nodes, ref_n)
    np.testing.assert_array_equal(scores, ref_s)
    if not os.path.exists(BOUNDS_SO):
        pytest.skip("libkoordgpu_bounds.so not built (python koordinator_amd/build.py --bounds)")
    bn, bs = _child_place(form, BOUNDS_SO)   # raises in the child (EngineError "bounds check: ...") on a violation
    np.testing.assert_array_equal(bn, ref_n)
    np.testing.assert_array_equal(bs, ref_s)


def test_sharded_cache_offset_bounds():
    """Two ranks on one GPU, shards [0, 1024) and [1024, 2048): the second rank's outcome cache is indexed from its
    column offset (k_eval_numa_cached's crow − col_begin, k_ncache_refresh's node − col_begin); product library
    and bounds build against the oracle."""
    ref_n, ref_s = _oracle("sharded_cache")
    for so in (None, BOUNDS_SO if os.path.exists(BOUNDS_SO) else None):
        outs = _sharded("sharded_cache", so)
        for n, s in outs:
            np.testing.assert_array_equal(np.asarray(n), ref_n)
            np.testing.assert_array_equal(np.asarray(s), ref_s)
