set -o pipefail
out=gpurun_out/r6zh; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -x -v -s --timeout 200 --timeout-method thread -k "other_hidden_width" > $out/hid.log 2>&1 || { tail -40 $out/hid.log; exit 1; }
grep -E "PASS|FAIL|passed|failed|fwd=" $out/hid.log | tail -6
