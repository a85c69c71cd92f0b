#!/bin/bash
# One GPU-box pass: parity tests, a bench line, the rocprof kernel trace + PMC passes, the SQ counter passes of
# k_eval3 (config 2) and k_eval_numa2 (config 3), and the placement kernel traces.
# Usage (from the repo root, on the GPU box): tools/gpu_check.sh <tag> [tests|bench|prof|sq|place|all]...
# PYTEST_ARGS adds pytest arguments (e.g. -k "not full_burst").
set -o pipefail
TAG=${1:-r01}
shift
WHAT=${*:-all}
has() { [[ " $WHAT " == *" all "* || " $WHAT " == *" $1 "* ]]; }
mkdir -p gpurun_out
export TMPDIR=/tmp
if has tests; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $PYTEST_ARGS \
    > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 1; }
  tail -3 gpurun_out/tests_$TAG.log
fi
if has bench; then
  timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { tail -30 gpurun_out/bench_$TAG.err; exit 2; }
  cat gpurun_out/bench_$TAG.json
fi
if has prof; then
  bash tools/profile.sh $TAG || exit 3
fi
if has sq; then
  bash tools/sqprof.sh ${TAG}_eval3 k_eval3 > gpurun_out/sq_${TAG}_eval3.txt 2>&1 || { tail -20 gpurun_out/sq_${TAG}_eval3.txt; exit 4; }
  SQPROF_BENCH="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-placement --c3-pods 1000 --c5-pods 0 --la-extra-pods 0" \
    bash tools/sqprof.sh ${TAG}_numa2 k_eval_numa2 > gpurun_out/sq_${TAG}_numa2.txt 2>&1 \
    || { tail -20 gpurun_out/sq_${TAG}_numa2.txt; exit 5; }
fi
if has place; then
  bash tools/gpu_place_prof.sh || exit 6
fi
echo gpu-check-done
