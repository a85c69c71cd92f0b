#!/bin/bash
# round-6 GPU session I: bench placement through kg_place_sharded over 8 loopback ranks on one GPU, then the whole GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --gpus 8 --backend loopback --steps 3 --warmup 1 > gpurun_out/r6i_loop8.json 2> gpurun_out/r6i_loop8.err
rc=$?
echo "loopback bench rc=$rc"; tail -c 1500 gpurun_out/r6i_loop8.json
if [ $rc -ne 0 ]; then tail -20 gpurun_out/r6i_loop8.err; exit $rc; fi
timeout -k 10 1000 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r6i_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r6i_tests.log
exit $rc
