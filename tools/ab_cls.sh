#!/bin/bash
# k_eval3 grid-shape A/B on the GPU box: config-2 matrix-mode kernel time for work-item targets
# (KG_CLS_TARGET_BLOCKS) and the two-stream kind launch (KG_CLS_CONCURRENT), interleaved twice.
# Usage: tools/ab_cls.sh <tag> "<target>:<concurrent>" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for r in 1 2; do
  for spec in "$@"; do
    tb=${spec%:*}; cc=${spec#*:}
    f=gpurun_out/abcls_${TAG}_${tb}_${cc}_$r.json
    KG_CLS_TARGET_BLOCKS=$tb KG_CLS_CONCURRENT=$cc timeout -k 10 180 $B > $f 2> gpurun_out/abcls_${TAG}.err || exit 2
    python -c "import json; d=json.load(open('$f')); print('$tb', '$cc', $r, d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
