#!/bin/bash
# round-6 GPU session M: Fit + LoadAware pass + NodeNUMAResource-only k_eval_numa2 (combine form): timing and parity
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for sec in c3_eq c3_distinct c5_matrix; do
  timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_named_resources_gpu.py tests/test_rsv_gpu.py tests/test_fullsize_place_gpu.py \
  tests/test_place_pipeline_gpu.py > gpurun_out/r6m_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r6m_tests.log
exit $rc
