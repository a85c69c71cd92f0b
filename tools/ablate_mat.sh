#!/bin/bash
# Matrix-mode bench (config 2, kernel time) of each measurement build in koordinator_amd/lib/variants, k_mat.
# Usage: tools/ablate_mat.sh <tag> <variant>[@eval3|@mat]...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for r in 1 2; do
  for spec in "$@"; do
    v=${spec%@*}; k=mat; [[ $spec == *@* ]] && k=${spec#*@}
    f=gpurun_out/abl_${TAG}_${v}_${k}_$r.json
    KG_ENGINE_SO=koordinator_amd/lib/variants/$v.so KG_MATRIX_KERNEL=$k timeout -k 10 180 $B > $f 2>gpurun_out/abl_${TAG}.err || exit 2
    python -c "import json; d=json.load(open('$f')); print('$v', '$k', $r, d['roofline']['kernel_ms'])"
  done
done
