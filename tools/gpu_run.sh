set -o pipefail
out=gpurun_out/r5l; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fly_fused.py -m gpu -x -v --timeout 200 --timeout-method thread > $out/fly.log 2>&1 && \
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf > $out/gputest.log 2>&1; rc=$?
grep -hE "FAILED|Error" $out/*.log | head -20
tail -3 $out/gputest.log $out/fly.log
exit $rc
