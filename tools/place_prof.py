"""One kg_place run (optional kernel forms as a third argument, e.g. 0x10 = FORM_NUMA_NO_CACHE) (config 2: 10k pods × 100k nodes; "c3": config 3, 1k pods, NodeNUMAResource; "c5": config 5,
20k pods of the Reservation + ElasticQuota burst) for rocprofv3 kernel traces of the placement path."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402

WHICH = sys.argv[1] if len(sys.argv) > 1 else "c2"
C3, C5 = WHICH == "c3", WHICH == "c5"
P = int(sys.argv[2]) if len(sys.argv) > 2 and int(sys.argv[2]) > 0 else (1_000 if C3 else 20_000 if C5 else 10_000)
FORMS = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0   # kg_set_forms bits (nat.FORM_*)
if C3:
    cl = synth.make_numa_cluster(100_000, P, seed=3)
elif C5:
    cl = synth.make_rsv_cluster(100_000, P, seed=5)
else:
    cl = synth.make_cluster(100_000, P, seed=2)
cfg = shipped_profile(plugins=("NodeResourcesFit", "LoadAwareScheduling", "Reservation", "ElasticQuota")) if C5 \
    else shipped_profile()
if C3:
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
rows = engine.build_node_rows(cfg, cl)
pods = engine.build_pod_rows(cfg, cl, np.arange(P))
with engine.Engine(cfg) as eng:
    eng.set_forms(FORMS)
    eng.load_snapshot(rows)
    if C5:
        eng.set_reservations(cl.rsv_arr)
        eng.set_quotas(cl.quota_arr)
    eng.set_pods(pods)
    eng.sync()
    t0 = time.perf_counter()
    nodes, scores = eng.place(cl.now_ns)
    dt = time.perf_counter() - t0
print(f"{'config3' if C3 else 'config5' if C5 else 'config2'} placement: {P} pods in {dt:.3f} s = {P / dt:.0f} pods/s", flush=True)
