#!/bin/bash
# round-6 GPU session C: section profiles (c2_distinct, c3_eq, c3_distinct, c5_matrix), placement A/B, bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/profile_sections.sh r6c c2_distinct c3_eq c3_distinct c5_matrix > gpurun_out/r6c_prof.log 2>&1
prc=$?
echo "profile rc=$prc"; tail -3 gpurun_out/r6c_prof.log
if [ $prc -ne 0 ]; then exit $prc; fi
for so in "" abl1 abl2; do
  for sec in c3_eq c3_distinct; do
    if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6;
    else timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6; fi
  done
done > gpurun_out/r6c_ablate.log 2>&1
cat gpurun_out/r6c_ablate.log
timeout -k 10 300 python -u tools/place_ab.py c2 --settings 0:16,1:16,1:24,1:32 --rounds 2 > gpurun_out/r6c_place_ab.log 2>&1 || exit 5
cat gpurun_out/r6c_place_ab.log
timeout -k 10 600 python -u bench.py > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err
echo "bench rc=$?"
