#!/bin/bash
# round-6 evidence session: headline profile (trace + PMC), section profiles, placement kernel stats, smoke, bench line
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r06_v1}
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/profile.sh $TAG > gpurun_out/${TAG}_prof.log 2>&1 || { echo "profile rc=$?"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
echo profile ok
bash tools/profile_sections.sh $TAG c2_distinct c3_eq c3_distinct c5_matrix > gpurun_out/${TAG}_sec.log 2>&1 || { echo "sections rc=$?"; tail -5 gpurun_out/${TAG}_sec.log; exit 2; }
echo sections ok
bash tools/gpu_place_prof.sh > gpurun_out/${TAG}_place.log 2>&1 || { echo "place rc=$?"; tail -5 gpurun_out/${TAG}_place.log; exit 3; }
grep placement gpurun_out/${TAG}_place.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${TAG}_smoke.log; exit 4; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
echo "bench rc=$rc"
tail -c 600 gpurun_out/${TAG}_bench.json
exit $rc
