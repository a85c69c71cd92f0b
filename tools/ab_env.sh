#!/bin/bash
# A/B of an engine launch switch on the GPU box: matrix-mode parity under the switch, then alternating
# bench runs (matrix mode only) with and without it.
# Usage: tools/ab_env.sh <tag> <VAR=value> [tests]
set -o pipefail
TAG=$1
SW=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $3 == tests ]]; then
  env $SW timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_rsv_gpu.py -k "not placement" \
    > gpurun_out/ab_${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/ab_${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/ab_${TAG}_tests.log
fi
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for i in 1 2; do
  timeout -k 10 180 $B > gpurun_out/ab_${TAG}_base$i.json 2>/dev/null || exit 2
  env $SW timeout -k 10 180 $B > gpurun_out/ab_${TAG}_sw$i.json 2>/dev/null || exit 3
done
for f in gpurun_out/ab_${TAG}_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); print('$f', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
