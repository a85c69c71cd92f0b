#!/bin/bash
# round-6 closing session: evidence (tools/gpu_r6_final.sh) then the whole GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r06_v3}
bash tools/gpu_r6_final.sh $TAG || exit $?
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_tests.log
exit $rc
