"""Debug helper: run one matrix eval on the GPU and dump the outputs for offline comparison."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from koordinator_amd import engine, synth
from koordinator_amd.config import make_config

cl = synth.make_cluster(5_000, 96, seed=11)
cfg = make_config()
idx = np.arange(96)
eng = engine.Engine(cfg)
eng.load_snapshot(engine.build_node_rows(cfg, cl))
eng.set_pods(engine.build_pod_rows(cfg, cl, idx))
res = eng.eval(cl.now_ns)
np.savez("gpurun_out/dump_matrix.npz", **res)
print("done")
