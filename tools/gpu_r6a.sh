#!/bin/bash
# round-6 GPU session A: loopback / bounds / pipeline / RCCL tests, then a short bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --maxfail=3 --timeout 300 --timeout-method thread \
  tests/test_loopback_gpu.py tests/test_bounds_gpu.py tests/test_place_pipeline_gpu.py tests/test_rccl_gpu.py \
  > gpurun_out/r6a_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -5 gpurun_out/r6a_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --c3-pods 0 --c5-pods 0 \
  --la-extra-pods 0 --no-distinct > gpurun_out/r6a_bench.json 2> gpurun_out/r6a_bench.err
rc2=$?
echo "bench rc=$rc2"
exit $rc
