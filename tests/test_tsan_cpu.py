"""ThreadSanitizer run of the oracle's threaded CPU baselines (the Parallelizer restatements kgo_eval_parallel
and kgo_schedule_parallel of oracle/koord_oracle.c, which bench.py times as cpu_baseline, and the threaded
Reservation + ElasticQuota cycle kgo_schedule2_parallel the full-size placement fixture is made with): tests/tsan_driver.c
and the oracle sources built with -fsanitize=thread into a standalone program (no Python in the instrumented
process), run on dumped clusters (the default profile, NodeNUMAResource with cpusets, Reservation + ElasticQuota),
checked against the
sequential cycle, and required to finish without a ThreadSanitizer report."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from bind_cases import make_bind_cluster
from koordinator_amd import _native as nat
from koordinator_amd import synth
from koordinator_amd.config import shipped_profile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "build", "tsan")


def _build():
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "oracle_tsan")
    srcs = [os.path.join(HERE, "tsan_driver.c"), os.path.join(ROOT, "oracle", "koord_oracle.c"),
            os.path.join(ROOT, "oracle", "cpu_accumulator.c")]
    r = subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fsanitize=thread", "-ffp-contract=off", "-I",
                        os.path.join(ROOT, "include"), *srcs, "-o", exe, "-lm", "-lpthread"],
                       capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("gcc -fsanitize=thread unavailable: " + r.stderr[-300:])
    return exe


def _dump(path, cfg, view, idx, now):
    arrays = list(view.c_view._keep)
    with open(path, "wb") as f:
        def put(a, dt):
            a = np.ascontiguousarray(a, dtype=dt).reshape(-1)
            f.write(np.array([dt.itemsize, len(a)], np.int64).tobytes())
            f.write(a.tobytes())
        put(np.asarray(cfg).reshape(1), nat.CONFIG)
        for a in arrays:
            put(a, a.dtype)
        put(np.asarray(idx, np.int32), np.dtype(np.int32))
        put(np.array([now], np.int64), np.dtype(np.int64))


@pytest.mark.parametrize("kind", ["default", "numa_cpuset", "rsv_quota"])
def test_oracle_parallel_baselines_under_tsan(kind, tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    exe = _build()
    if kind == "default":
        cl = synth.make_cluster(1500, 48, seed=31)
        cfg, view, idx, now = shipped_profile(), cl, np.arange(48), cl.now_ns
    elif kind == "rsv_quota":
        cl = synth.make_rsv_cluster(1200, 60, seed=33, rsv_node_frac=0.05, quota_ratio=0.6, affinity_frac=0.5,
                                    quota_tree=True)
        cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota"),
                              eq_check_parent_quota=1)
        view, idx, now = cl, np.arange(60), cl.now_ns
    else:
        cl, view, idx = make_bind_cluster(200, 40, 32)
        cfg = shipped_profile()
        cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
        now = cl.now_ns
    path = str(tmp_path / "view.bin")
    _dump(path, cfg, view, idx, now)
    r = subprocess.run([exe, path], capture_output=True, text=True, timeout=600,
                       env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1:exitcode=66"))
    assert r.returncode == 0, r.stdout[-1000:] + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "tsan workload ok" in r.stdout
