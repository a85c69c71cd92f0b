set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_new.log 2>&1 || { tail -30 gpurun_out/t_new.log; exit 1; }
tail -1 gpurun_out/t_new.log
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-placement --no-cpu-baseline --c3-pods 0 --c5-pods 0 > gpurun_out/b_new.json 2>gpurun_out/b_new.err || { tail -20 gpurun_out/b_new.err; exit 2; }
python -c "import json;d=json.load(open('gpurun_out/b_new.json'));print('new', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
