#!/bin/bash
# round-6 GPU session J: reciprocal quotients in the NodeNUMAResource scores (c3 sections) + NUMA parity
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sec in c3_eq c3_distinct; do
  timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_fullsize_place_gpu.py > gpurun_out/r6j_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6j_tests.log
exit $rc
