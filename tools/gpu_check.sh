#!/bin/bash
# One GPU-box pass: parity tests, a bench line, then the rocprof kernel trace + PMC passes.
# Usage (from the repo root, on the GPU box): tools/gpu_check.sh <tag> [tests|bench|prof|all]
set -o pipefail
TAG=${1:-r01}
WHAT=${2:-all}
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ $WHAT == all || $WHAT == tests ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { tail -30 gpurun_out/bench_$TAG.err; exit 2; }
  cat gpurun_out/bench_$TAG.json
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  bash tools/profile.sh $TAG || exit 3
fi
echo gpu-check-done
