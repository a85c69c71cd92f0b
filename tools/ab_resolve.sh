#!/bin/bash
# k_resolve barrier A/B: placement parity under the variant, then interleaved config-2 / config-3 placement runs.
# Usage: tools/ab_resolve.sh <variant>
set -o pipefail
V=$1
mkdir -p gpurun_out
export TMPDIR=/tmp
SO=koordinator_amd/lib/variants/$V.so
KG_ENGINE_SO=$SO timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_fullsize_place_gpu.py tests/test_rsv_gpu.py tests/test_numa_gpu.py -k "place or config5" \
  > gpurun_out/abres_${V}_tests.log 2>&1 || { tail -30 gpurun_out/abres_${V}_tests.log; exit 1; }
tail -1 gpurun_out/abres_${V}_tests.log
for r in 1 2; do
  for so in koordinator_amd/lib/libkoordgpu.so $SO; do
    KG_ENGINE_SO=$so timeout -k 10 120 python tools/place_prof.py | sed "s|^|$(basename $so) |" || exit 2
    KG_ENGINE_SO=$so timeout -k 10 120 python tools/place_prof.py c3 | sed "s|^|$(basename $so) |" || exit 3
  done
done
