#!/bin/bash
# Round-3 final pass: parity subset (fold, debug dump), bench line, rocprofv3 trace + PMC, waves-per-SIMD A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/par_r03p.log 2>&1 || { tail -30 gpurun_out/par_r03p.log; exit 1; }
tail -1 gpurun_out/par_r03p.log
bash tools/gpu_check.sh r03p bench || exit 2
bash tools/profile.sh r03p || exit 3
bash tools/ab_so.sh r03w wpe8 wpe5 --notests || exit 4
