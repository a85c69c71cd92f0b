#!/bin/bash
# Round-3 NUMA check: parity of the queued k_eval_numa2 / numa2 placement chunks, config-3 placement A/B
# (k_eval_numa_chunk vs k_eval_numa2 chunks), matrix-mode kernel time.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py \
  tests/test_bind_gpu.py tests/test_fullsize_place_gpu.py > gpurun_out/par_r03l.log 2>&1 || { tail -30 gpurun_out/par_r03l.log; exit 1; }
tail -2 gpurun_out/par_r03l.log
for r in 1 2; do
  for cp in 16 0; do
    KG_NUMA_CHUNK_PODS=$cp timeout -k 10 120 python tools/place_prof.py c3 | sed "s/^/chunk_pods=$cp /" || exit 3
  done
done
bash tools/ablate_numa.sh r03l base || exit 4
