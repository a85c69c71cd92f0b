#!/bin/bash
# Kernel trace + SQ counter passes (one counter group per rocprofv3 run) over the matrix-mode bench,
# GPU box only.  Usage: tools/sqprof.sh <tag> [kernel-name substring]   → gpurun_out/sq_<tag>/...
set -o pipefail
TAG=${1:-x}
KNAME=${2:-k_eval}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH=${SQPROF_BENCH:-"python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0 --la-extra-pods 0"}
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $BENCH > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 9; }
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_WR"
P3="SQ_BUSY_CYCLES SQ_WAVES SQ_LEVEL_WAVES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- $BENCH > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit $i; }
done
python - "$OUT" "$KNAME" <<'PY'
import csv, glob, sys, collections
out, kname = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c) in sorted(acc):
    v = acc[(k, c)]
    print(f"{k:60s} {c:28s} {sum(v)/len(v):16.0f}")
for f in glob.glob(out + "/trace/**/*kernel_stats.csv", recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print(r["Name"][:90], r["Calls"], r["AverageNs"], r["Percentage"])
PY
