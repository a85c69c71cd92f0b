#!/bin/bash
# A/B of the matrix-mode kernel with planes (KG_MATRIX_KERNEL=eval3 | mat) on the GPU box: parity of the
# matrix-mode tests under k_mat, then interleaved config-2 bench runs (matrix mode only).
# Usage: tools/ab_mat.sh <tag> [notests]
set -o pipefail
TAG=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $2 != notests ]]; then
  KG_MATRIX_KERNEL=mat timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_rsv_gpu.py tests/test_la_extra_gpu.py \
    tests/test_numa_gpu.py -k "not placement" > gpurun_out/abmat_${TAG}_tests.log 2>&1 \
    || { tail -30 gpurun_out/abmat_${TAG}_tests.log; exit 1; }
  tail -2 gpurun_out/abmat_${TAG}_tests.log
fi
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for r in 1 2; do
  for k in eval3 mat; do
    f=gpurun_out/abmat_${TAG}_${k}_$r.json
    KG_MATRIX_KERNEL=$k timeout -k 10 180 $B > $f 2> gpurun_out/abmat_${TAG}_${k}_$r.err || exit 2
    python -c "import json; d=json.load(open('$f')); print('$k', $r, d['roofline']['kernel_ms'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
