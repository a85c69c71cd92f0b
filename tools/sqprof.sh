#!/bin/bash
# SQ counter passes over the matrix-mode bench (one pass per rocprofv3 run), GPU box only.
# Usage: tools/sqprof.sh <tag>   → gpurun_out/sq_<tag>/<pass>/...
set -o pipefail
TAG=${1:-x}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-placement"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INST_CYCLES_VMEM_WR"
P3="SQ_BUSY_CYCLES SQ_WAVES SQ_LEVEL_WAVES SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
P4="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- $BENCH > $OUT/p$i.log 2>&1 || { tail -5 $OUT/p$i.log; exit $i; }
done
python - "$OUT" <<'EOF'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_eval" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:32s} {sum(v)/len(v):16.0f}")
EOF
