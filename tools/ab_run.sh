# GPU check of the current tree: fly / repeats tests, then a fly-mode bench line
mkdir -p gpurun_out/ab3
timeout -k 10 400 python -u -m pytest tests/test_gpu_fly.py tests/test_gpu_configs.py tests/test_gpu_micro.py tests/test_gpu_dashboard.py tests/test_gpu_dp.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3/tests.log 2>&1 || { tail -40 gpurun_out/ab3/tests.log; exit 1; }
tail -1 gpurun_out/ab3/tests.log
timeout -k 10 200 python bench.py --no-cpu-baseline --sampling fly > gpurun_out/ab3/c2_fly.json 2>gpurun_out/ab3/c2_fly.err || exit 1
echo ok
