import ctypes, sys, time
import numpy as np
sys.path.insert(0, ".")
from koordinator_amd import _native as nat, engine, synth
from koordinator_amd.config import shipped_profile
cl = synth.make_cluster(100_000, 10_000, seed=2)
cfg = shipped_profile()
rows = engine.build_node_rows(cfg, cl)
pods = engine.build_pod_rows(cfg, cl, np.arange(10_000))
with engine.Engine(cfg) as eng:
    eng.load_snapshot(rows); eng.set_pods(pods); eng.sync()
    t0 = time.perf_counter(); eng.place(cl.now_ns); dt = time.perf_counter() - t0
out = (ctypes.c_ulonglong * 16)()
nat.lib().kg_debug_rprof(out)
v = np.array(list(out)[:8], dtype=np.float64) * 10 / 10_000   # 100 MHz ticks -> ns per pod
print("place s", dt, "ns per pod by phase:", [round(x) for x in v], "sum", round(v.sum()))
