#!/bin/bash
# rocprofv3 kernel trace + SQ / HBM PMC passes of single bench sections (tools/section_run.py), one GPU.
# Usage: tools/profile_sections.sh <tag> <section>...   (run on the GPU box from the repo root)
set -o pipefail
TAG=$1
shift
export TMPDIR=/tmp
for S in "$@"; do
  OUT=gpurun_out/sec_${TAG}/$S
  mkdir -p $OUT
  RUN="python tools/section_run.py $S --reps 5"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $RUN > $OUT/trace.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $OUT/pmc_sq -o pmc_sq --output-format csv -- $RUN > $OUT/pmc_sq.log 2>&1 || exit 2
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc_fetch --output-format csv -- $RUN > $OUT/pmc_fetch.log 2>&1 || exit 3
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc_write --output-format csv -- $RUN > $OUT/pmc_write.log 2>&1 || exit 4
  echo "section $S profiled"
done
echo profile-sections-done
