"""Per-pod phase costs of k_resolve (GPU box, measurement build with -DKG_RESOLVE_TIMING):
    KG_ENGINE_SO=ab/rtime/libkoordgpu.so python tools/resolve_timing.py [config2|config3|config5] [pods]
Phases (thread 0's s_memtime, shader-clock cycles): 1→2 tile scan + touched / previous-chunk re-scores (up to the
first barrier), 2→3 rescans + wave max + barrier, 3→4 block max → the committed row staged (+ zone commit),
4→5 Reserve parts, 5→6 flags + the pod's last barrier."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from koordinator_amd import _native as nat  # noqa: E402
from koordinator_amd import engine, synth  # noqa: E402
from koordinator_amd.config import shipped_profile  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config2"
P = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
cfg = shipped_profile()
if which == "config3":
    cl = synth.make_numa_cluster(100_000, P, seed=3)
    cfg["enabled_plugins"] |= nat.PLUGIN_NUMA
else:
    cl = synth.make_cluster(100_000, P, seed=2)
with engine.Engine(cfg) as eng:
    eng.load_snapshot(engine.build_node_rows(cfg, cl))
    eng.set_pods(engine.build_pod_rows(cfg, cl, np.arange(P)))
    eng.sync()
    t0 = time.perf_counter()
    nodes, _ = eng.place(cl.now_ns)
    dt = time.perf_counter() - t0
L = nat.lib()
f = L.kg_debug_resolve_times
f.restype = ctypes.c_int32
f.argtypes = [ctypes.c_void_p, ctypes.c_int32]
buf = np.zeros((P, 16), np.uint64)
k = f(buf.ctypes.data, P)
t = buf[:k].astype(np.int64)
ok = (t[:, 6] > 0) & (t[:, 1] > 0)
d = np.diff(t[ok][:, 1:7], axis=1)
print(f"{which}: {P} pods, {P / dt:.0f} pods/s, {int(ok.sum())} timed pods")
for i, name in enumerate(["scan+rescore", "rescan+wavemax", "blockmax+row", "reserve parts", "flags+sync"]):
    print(f"  {name:16s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f} cycles")
tt = t[ok]
fit1 = tt[:, 7] - tt[:, 4]
la0 = tt[:, 0] - tt[:, 4]
print(f"  reserve: Fit part (memory) done after median {np.median(fit1):8.0f}, LoadAware part (cpu) after "
      f"{np.median(la0):8.0f} cycles")
for slot, name in ((9, "thread 0 after its tile"), (11, "thread 97 after its tile"), (8, "touched re-score (thread 128)"),
                   (10, "next pod's row prefetched (thread 511)")):
    x = tt[:, slot] - tt[:, 1]
    print(f"  scan: {name:40s} median {np.median(x[tt[:, slot] > 0]) if (tt[:, slot] > 0).any() else float('nan'):8.0f}")
tot = t[ok][:, 6] - t[ok][:, 1]
print(f"  total per pod   median {np.median(tot):8.0f}  mean {tot.mean():8.0f}")
nxt = t[ok][1:, 1] - t[ok][:-1, 6]
print(f"  gap to next pod (incl. launches between chunks) median {np.median(nxt):8.0f}")
