#!/bin/bash
# A/B of engine builds (tools/build_variants.sh) on the GPU box: matrix-mode parity under each variant,
# then interleaved config-2 bench runs (matrix mode only) of the default library and every variant.
# Usage: tools/ab_so.sh <tag> <variant> ... [--notests]
set -o pipefail
TAG=$1; shift
VARS=(); TESTS=1
for v in "$@"; do [[ $v == --notests ]] && TESTS=0 || VARS+=("$v"); done
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $TESTS == 1 ]]; then
  for v in "${VARS[@]}"; do
    KG_ENGINE_SO=koordinator_amd/lib/variants/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
      --timeout-method thread tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_rsv_gpu.py -k "not placement" \
      > gpurun_out/abso_${TAG}_${v}_tests.log 2>&1 || { tail -30 gpurun_out/abso_${TAG}_${v}_tests.log; exit 1; }
    echo "$v: $(tail -1 gpurun_out/abso_${TAG}_${v}_tests.log)"
  done
fi
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for r in 1 2 3; do
  for v in base "${VARS[@]}"; do
    so=koordinator_amd/lib/libkoordgpu.so; [[ $v != base ]] && so=koordinator_amd/lib/variants/$v.so
    f=gpurun_out/abso_${TAG}_${v}_$r.json
    KG_ENGINE_SO=$so timeout -k 10 180 $B > $f 2> gpurun_out/abso_${TAG}_${v}_$r.err || exit 2
    python -c "import json; d=json.load(open('$f')); print('$v', $r, d['roofline']['kernel_ms'], d['ms_per_step'])"
  done
done
