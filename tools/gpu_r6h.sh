#!/bin/bash
# round-6 GPU session H: k_eval_numa2 split after the single-zone path (product / base only / every pair single-zone)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for so in "" abl2 abl3; do
  for sec in c3_eq c3_distinct; do
    echo -n "[$so] "
    if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6;
    else timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6; fi
  done
done 2>&1 | grep -v amdgpu.ids
OUT=gpurun_out/sec_r6h/c3_eq
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python tools/section_run.py c3_eq --reps 5 > $OUT/trace.log 2>&1 || exit 2
echo traced
