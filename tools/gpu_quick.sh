#!/bin/bash
# quick GPU timing session: section passes and placement rates (no profiler), then optional pytest targets
# usage: tools/gpu_quick.sh <tag> [pytest args...]
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; shift
mkdir -p gpurun_out
{
for sec in c2_distinct c3_eq c3_distinct c5_matrix; do
  timeout -k 10 120 python -u tools/section_run.py $sec --reps 5 || exit 6
done
timeout -k 10 200 python -u tools/place_ab.py c2 --settings 0:16 --rounds 2 || exit 7
timeout -k 10 200 python -u tools/place_ab.py c3 --settings 0:16 --rounds 2 || exit 8
timeout -k 10 200 python -u tools/place_ab.py c5 --settings 0:16 --rounds 1 || exit 9
} > gpurun_out/${TAG}_quick.log 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/${TAG}_quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -q --maxfail=5 --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  tail -5 gpurun_out/${TAG}_tests.log
fi
exit $rc
