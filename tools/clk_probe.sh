set -o pipefail
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-placement --c3-pods 0 --c5-pods 0"
for v in lib lib/ab/1 lib/ab/16; do
  t=$(echo $v | tr / _)
  KG_ENGINE_SO=koordinator_amd/$v/libkoordgpu.so timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES -d gpurun_out/clk/$t -o p --output-format csv -- $B > gpurun_out/clk/$t.log 2>&1 || { tail -5 gpurun_out/clk/$t.log; exit 1; }
  KG_ENGINE_SO=koordinator_amd/$v/libkoordgpu.so timeout -k 10 90 rocprofv3 --kernel-trace --stats -d gpurun_out/clk/${t}_tr -o t --output-format csv -- $B > gpurun_out/clk/${t}_tr.log 2>&1 || exit 2
done
python - <<'PY'
import csv, glob, collections
for t in ["lib", "lib_ab_1", "lib_ab_16"]:
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/clk/{t}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_eval3" in r["Kernel_Name"] and ", true>" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = None
    for f in glob.glob(f"gpurun_out/clk/{t}_tr/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_eval3" in r["Name"] and ", true>" in r["Name"]:
                dur = float(r["AverageNs"])
    g = sum(acc["GRBM_GUI_ACTIVE"]) / len(acc["GRBM_GUI_ACTIVE"])
    print(t, "dur_ns", dur, "GRBM", g, "GHz(GRBM/8/dur)", g / 8 / dur if dur else None)
PY
