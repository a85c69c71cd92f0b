#!/bin/bash
# round-6 GPU session D: k_eval_numa2 whole-segment flush A/B (product FL=32 vs variant), WRITE_SIZE of c3_distinct,
# NUMA parity tests
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for so in "" fl16; do
  for sec in c3_eq c3_distinct; do
    if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6;
    else timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6; fi
  done
done > gpurun_out/r6d_ab.log 2>&1
cat gpurun_out/r6d_ab.log | grep -v amdgpu.ids
OUT=gpurun_out/sec_r6d/c3_distinct
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python tools/section_run.py c3_distinct --reps 5 > $OUT/trace.log 2>&1 || exit 2
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc_write --output-format csv -- python tools/section_run.py c3_distinct --reps 5 > $OUT/pmc_write.log 2>&1 || exit 3
echo profiled
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_numa_gpu.py tests/test_parity_gpu.py \
  tests/test_fullsize_gpu.py tests/test_fullsize_place_gpu.py tests/test_named_resources_gpu.py > gpurun_out/r6d_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6d_tests.log
exit $rc
