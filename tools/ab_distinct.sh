#!/bin/bash
# A/B of engine builds on the config2_distinct section (the per-pair k_eval3 plain path), GPU box:
# tools/ab_distinct.sh <tag> <so-dir>...   (interleaved, twice each)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
  for d in "$@"; do
    KG_ENGINE_SO=$d/libkoordgpu.so timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-placement --no-host-outputs --steps 4 \
      --c3-pods 0 --c5-pods 0 --la-extra-pods 0 > gpurun_out/abd_${TAG}.json 2> gpurun_out/abd_${TAG}.err || { tail -20 gpurun_out/abd_${TAG}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/abd_${TAG}.json').read().strip().splitlines()[-1]); print('$d', 'dup', d['roofline']['kernel_ms'], 'distinct', d['config2_distinct']['kernel_ms'])"
  done
done
