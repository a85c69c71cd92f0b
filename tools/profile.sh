#!/bin/bash
# Kernel trace + PMC passes for the matrix-mode bench (run on the GPU box from the repo root).
# Usage: tools/profile.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-placement --no-distinct --no-host-outputs --c3-pods 0 --c5-pods 0 --la-extra-pods 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $BENCH > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_sq -o pmc_sq --output-format csv -- $BENCH > $OUT/pmc_sq.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc_fetch --output-format csv -- $BENCH > $OUT/pmc_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_write -o pmc_write --output-format csv -- $BENCH > $OUT/pmc_write.log 2>&1 || exit 4
echo profile-done
