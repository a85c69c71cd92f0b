#!/bin/bash
# round-6 GPU session F: k_eval_numa2 variants (base / launder / launder without fill+enumeration / lite fill)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for so in base lnd lnd2 lite; do
  for sec in c3_eq c3_distinct; do
    echo -n "$so "
    KG_ENGINE_SO=koordinator_amd/lib/libkoordgpu_$so.so timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6
  done
done 2>&1 | grep -v amdgpu.ids
