#!/bin/bash
# round-6 GPU session G: single-zone NUMA path + row prefetch in k_eval_numa2 (product vs the r6 base), NUMA parity
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for so in base ""; do
  for sec in c3_eq c3_distinct; do
    echo -n "[$so] "
    if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6;
    else timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6; fi
  done
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_fullsize_place_gpu.py tests/test_named_resources_gpu.py > gpurun_out/r6g_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6g_tests.log
exit $rc
