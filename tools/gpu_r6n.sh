#!/bin/bash
# round-6 GPU session N: k_eval_numa2 at 4 waves per SIMD (variant) against the product
cd "$GRAFT_REPO_ROOT" || exit 1
for so in "" wpe4 ""; do
  for sec in c3_eq c3_distinct; do
    echo -n "[$so] "
    if [ -n "$so" ]; then KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6;
    else timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6; fi
  done
done 2>&1 | grep -v amdgpu.ids
