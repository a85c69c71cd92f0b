#!/bin/bash
# One GPU-box iteration on the hot path: the matrix-mode parity tests, a bench line (no CPU baseline), and
# the SQ counter passes of k_eval3.  Usage (GPU box, repo root): tools/gpu_iter.sh <tag> [extra pytest args]
set -o pipefail
TAG=${1:-x}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 200 --timeout-method thread "$@" \
  > gpurun_out/${TAG}_parity.log 2>&1 || { tail -30 gpurun_out/${TAG}_parity.log; exit 1; }
tail -2 gpurun_out/${TAG}_parity.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --c3-pods 0 --c5-pods 0 --la-extra-pods 0 > gpurun_out/${TAG}_bench.json \
  2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 2; }
python - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms_per_step", d["ms_per_step"], "kernel_ms", r["kernel_ms"], "frac", r["frac"],
      "place", d.get("placement", {}).get("pods_placed_per_s"))
PY
bash tools/sqprof.sh $TAG k_eval3 > gpurun_out/${TAG}_sq.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sq.txt; exit 3; }
grep -E 'SQ_INSTS_VALU |SQ_INSTS_SALU |SQ_WAIT_INST_ANY|SQ_WAVE_CYCLES|SQ_LDS_BANK|GRBM_GUI|SQ_ACTIVE_INST_VALU|k_eval3<' gpurun_out/${TAG}_sq.txt | cut -c1-20,60-
