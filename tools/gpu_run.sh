set -o pipefail
out=gpurun_out/r6j; mkdir -p $out
PINSAGE_KW_WAVES=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_wgrad.py -x -q --timeout 100 --timeout-method thread > $out/wreg.log 2>&1 || { tail -30 $out/wreg.log; exit 1; }
tail -1 $out/wreg.log
timeout -k 10 200 python -u tools/wgrad_bench.py > $out/wb.log 2>&1 || { tail -30 $out/wb.log; exit 1; }
grep dQ0 $out/wb.log; grep dW0 $out/wb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_c5.py -x -v -s --timeout 550 --timeout-method thread > $out/c5.log 2>&1 || { tail -40 $out/c5.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" $out/c5.log | tail -3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread --deselect tests/test_gpu_c5.py > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
grep -o "'grad_normrel_B_max': [0-9.e-]*" $out/gputest.log | sort -t: -k2 -g | tail -2
PINSAGE_TEST_CSR_FORK=1 PINSAGE_SEGV_BT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q -s --timeout 200 --timeout-method thread -k "forked" > $out/t2.log 2>&1; echo "forked rc $?"; grep -A40 "segv_bt" $out/t2.log | head -50; tail -2 $out/t2.log
