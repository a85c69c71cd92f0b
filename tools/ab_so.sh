#!/bin/bash
# A/B of engine builds / switches on the matrix-mode bench (GPU box): tools/ab_so.sh <tag> <spec>... where a spec is
# <so-dir>[:VAR=value[,VAR=value]] (koordinator_amd/lib = the default build); runs are interleaved, three times each.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for rep in 1 2 3; do
  for spec in "$@"; do
    d=${spec%%:*}; envs=""
    [[ $spec == *:* ]] && envs=${spec#*:}
    env ${envs//,/ } KG_ENGINE_SO=$d/libkoordgpu.so timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-placement --no-distinct --no-host-outputs \
      --c3-pods 0 --c5-pods 0 --la-extra-pods 0 > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { tail -20 gpurun_out/ab_${TAG}.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${TAG}.json').read().strip().splitlines()[-1]); print('$spec', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
