#!/bin/bash
# round-6 GPU session B: the GPU suite after the 12-resource change (the full-size placement fixture is being
# regenerated: its test is left out), section profiles, the default bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread -m gpu tests \
  --ignore=tests/test_fullsize_place_gpu.py > gpurun_out/r6b_tests.log 2>&1
rc=$?
echo "tests rc=$rc"
tail -15 gpurun_out/r6b_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
tools/profile_sections.sh r6b c2_distinct c3_eq c3_distinct c5_matrix > gpurun_out/r6b_prof.log 2>&1
prc=$?
echo "profile rc=$prc"; tail -3 gpurun_out/r6b_prof.log
if [ $prc -ne 0 ]; then exit $prc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r6b_bench.json 2> gpurun_out/r6b_bench.err
echo "bench rc=$?"
exit $rc
