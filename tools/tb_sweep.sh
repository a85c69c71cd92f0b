for tb in 1024 2048 4096 8192; do
  KG_TARGET_BLOCKS=$tb timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-placement > gpurun_out/tb_$tb.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/tb_$tb.json')); print('tb', $tb, d['roofline']['kernel_ms'])"
done
