set -o pipefail
out=gpurun_out/r6c; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_micro.py tests/test_gpu_dashboard.py -x -q -s --timeout 300 --timeout-method thread > $out/norm.log 2>&1 || { tail -60 $out/norm.log; exit 1; }
tail -1 $out/norm.log
grep -o "'grad_normrel_B_max': [0-9.e-]*" $out/norm.log | sort -t: -k2 -g | tail -3
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py -x -v -s --timeout 500 --timeout-method thread > $out/c5.log 2>&1 || { tail -60 $out/c5.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $out/c5.log | tail -3
