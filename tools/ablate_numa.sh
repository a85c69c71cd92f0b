#!/bin/bash
# Config-3 matrix-mode kernel time (k_eval_numa2, 1k pods × 100k nodes) of measurement builds in
# koordinator_amd/lib/variants (tools/build_variants.sh with -DKG_NUMA_ABLATE=...), interleaved twice.
# Usage: tools/ablate_numa.sh <tag> <variant>...   (a variant VAR=value runs the default build with that env)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-placement --c3-pods 1000 --c3-large-pods 0 --c5-pods 0 --pods 64"
for r in 1 2; do
  for v in "$@"; do
    so=koordinator_amd/lib/variants/$v.so; envv=KG_NONE=0
    [[ $v == base ]] && so=koordinator_amd/lib/libkoordgpu.so
    [[ $v == *=* ]] && { so=koordinator_amd/lib/libkoordgpu.so; envv=$v; }
    f=gpurun_out/ablnuma_${TAG}_${v}_$r.json
    env $envv KG_ENGINE_SO=$so timeout -k 10 300 $B > $f 2>gpurun_out/ablnuma_${TAG}.err || exit 2
    python -c "import json; d=json.load(open('$f')); print('$v', $r, d['config3']['kernel_ms'])"
  done
done
