#!/bin/bash
# round-6 GPU session R: exact quotients by kg_qdiv in the exact pair path (Reservation restore, slow nodes):
# config-5 matrix and placement, Reservation / parity / full-size placement suites
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for so in base ""; do
  echo -n "[$so] "
  if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py c5_matrix --reps 5 || exit 6;
  else timeout -k 10 120 python -u tools/section_run.py c5_matrix --reps 5 || exit 6; fi
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/place_ab.py c5 --settings 0:16 --rounds 2 2>&1 | grep -v amdgpu.ids || exit 5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rsv_gpu.py tests/test_parity_gpu.py \
  tests/test_fullsize_place_gpu.py tests/test_named_resources_gpu.py tests/test_la_extra_gpu.py tests/test_numa_gpu.py > gpurun_out/r6r_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6r_tests.log
exit $rc
