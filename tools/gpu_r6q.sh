#!/bin/bash
# round-6 GPU session Q: the single-zone NodeNUMAResource path in the per-pair kernels (resolve re-scores, cache
# refresh, placement chunks): config-3 placement rate and NUMA placement parity
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/place_ab.py c3 --settings 0:16 --rounds 3 2>&1 | grep -v amdgpu.ids || exit 5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py tests/test_fullsize_place_gpu.py \
  tests/test_place_pipeline_gpu.py tests/test_bounds_gpu.py tests/test_loopback_gpu.py tests/test_bind_gpu.py > gpurun_out/r6q_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6q_tests.log
exit $rc
