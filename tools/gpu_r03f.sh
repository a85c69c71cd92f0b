#!/bin/bash
# Round-3 check: parity of the pipelined placement / concurrent kinds, placement A/B, NUMA ablations.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py \
  tests/test_numa_gpu.py tests/test_bind_gpu.py tests/test_fullsize_place_gpu.py tests/test_dist.py \
  > gpurun_out/par_r03f.log 2>&1 || { tail -30 gpurun_out/par_r03f.log; exit 1; }
tail -2 gpurun_out/par_r03f.log
for r in 1 2; do
  for pp in 1 0; do
    KG_PLACE_PIPELINE=$pp timeout -k 10 120 python tools/place_prof.py | sed "s/^/pipeline=$pp /" || exit 2
    KG_PLACE_PIPELINE=$pp timeout -k 10 120 python tools/place_prof.py c3 | sed "s/^/pipeline=$pp /" || exit 3
  done
done
bash tools/ablate_numa.sh r03f base na1 na2 na4 || exit 4
