#!/bin/bash
# Round-3: full GPU suite at the uniform-slot fold build, then the fold A/B on config 2 (matrix mode).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_r03m.log 2>&1 || { tail -30 gpurun_out/tests_r03m.log; exit 1; }
tail -2 gpurun_out/tests_r03m.log
bash tools/ab_env.sh fold KG_CLS_FOLD_UNIFORM=0 || exit 2
