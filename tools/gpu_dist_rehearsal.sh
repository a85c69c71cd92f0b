#!/bin/bash
# GPU box: N>1 rehearsal of bench.py on one GPU (2 ranks on cuda:0 over gloo) beside the one-GPU line of the
# same workload, then config4 on one GPU.
set -o pipefail
mkdir -p gpurun_out
P=${PODS:-2000}
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --c3-pods 0 --c5-pods 0 --la-extra-pods 0 --pods $P \
  > gpurun_out/dist1.json 2> gpurun_out/dist1.err || { tail -30 gpurun_out/dist1.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline --c3-pods 0 \
  --c5-pods 0 --pods $P > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -30 gpurun_out/dist2.err; exit 2; }
python - <<'PY'
import json
for f in ("gpurun_out/dist1.json", "gpurun_out/dist2.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["n_gpus"], "evals/s", d["value"], "placement", d.get("placement", {}).get("pods_placed_per_s"),
          d.get("placement", {}).get("mode"))
PY
if [ "${C4:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py --scaling config4 --steps 3 --warmup 1 --no-cpu-baseline --no-placement \
    --c3-pods 0 --c5-pods 0 --la-extra-pods 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -30 gpurun_out/c4.err; exit 3; }
  tail -c 1500 gpurun_out/c4.json
fi
