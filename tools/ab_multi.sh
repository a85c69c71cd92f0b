#!/bin/bash
# Matrix-mode bench (config 2, kernel time only) under several settings of one engine switch, two
# interleaved rounds.  Usage: tools/ab_multi.sh <tag> <VAR> <value>... ("-" = unset)
set -o pipefail
TAG=$1
VAR=$2
shift 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for r in 1 2; do
  for v in "$@"; do
    f=gpurun_out/abm_${TAG}_${v//,/_}_$r.json
    if [[ $v == - ]]; then
      timeout -k 10 180 $B > $f 2>/dev/null || exit 2
    else
      env $VAR=$v timeout -k 10 180 $B > $f 2>/dev/null || exit 3
    fi
    python -c "import json; d=json.load(open('$f')); print('$v', $r, d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
