#!/bin/bash
# GPU box: N>1 rehearsal of bench.py on one GPU (2 ranks on cuda:0 over gloo), then config4 on one GPU.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline --c3-pods 0 \
  --c5-pods 0 --pods 2000 > gpurun_out/dist2.json 2> gpurun_out/dist2.err || { tail -30 gpurun_out/dist2.err; exit 1; }
tail -c 1500 gpurun_out/dist2.json
timeout -k 10 300 python bench.py --scaling config4 --steps 3 --warmup 1 --no-cpu-baseline --no-placement \
  --c3-pods 0 --c5-pods 0 > gpurun_out/c4.json 2> gpurun_out/c4.err || { tail -30 gpurun_out/c4.err; exit 2; }
tail -c 1500 gpurun_out/c4.json
