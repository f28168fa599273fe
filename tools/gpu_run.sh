set -o pipefail
out=gpurun_out/r5aa; R=$(pwd); mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_micro.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $out/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" $out/t.log | grep -v "^E  *$" | tail -n 30
exit $rc
