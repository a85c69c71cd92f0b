#!/bin/bash
# TEMP: k_eval time with parts of the hot loop switched off (KG_ABLATE bits), GPU box only.
set -o pipefail
mkdir -p gpurun_out
for v in ${@:-0 1 2 4 8 3 7 15}; do
  KG_ABLATE=$v timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-placement \
    > gpurun_out/ablate_$v.json 2> gpurun_out/ablate_$v.err || { tail -20 gpurun_out/ablate_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ablate_$v.json')); print('ablate', $v, d['roofline']['kernel_ms'], d['ms_per_step'])"
done
