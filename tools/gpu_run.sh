set -o pipefail
out=gpurun_out/r5e; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
tail -3 $out/gputest.log
