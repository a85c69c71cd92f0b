#!/bin/bash
# round-6 GPU session B1: the GPU suite after the 12-resource change (the full-size placement fixture is being
# regenerated: its test is left out)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests \
  --ignore=tests/test_fullsize_place_gpu.py > gpurun_out/r6b_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -15 gpurun_out/r6b_tests.log
exit $rc
