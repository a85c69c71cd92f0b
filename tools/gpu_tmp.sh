set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py tests/test_rsv_gpu.py tests/test_numa_gpu.py tests/test_dist.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_resolve.log 2>&1 || { tail -30 gpurun_out/t_resolve.log; exit 1; }
tail -2 gpurun_out/t_resolve.log
timeout -k 10 300 python tools/place_sweep.py 10000 > gpurun_out/sweep_c2.log 2>&1 || { tail gpurun_out/sweep_c2.log; exit 2; }
cat gpurun_out/sweep_c2.log
bash tools/gpu_place_prof.sh
