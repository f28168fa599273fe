set -o pipefail
out=gpurun_out/r6s; mkdir -p $out
PINSAGE_WGRAD_PLANES=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants_train_alike and (PLANES or FORK_PLAN)" > $out/var.log 2>&1 || { tail -30 $out/var.log; exit 1; }
tail -1 $out/var.log
PINSAGE_WGRAD_PLANES=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "train_step or model" > $out/par.log 2>&1 || { tail -30 $out/par.log; exit 1; }
tail -1 $out/par.log
bash tools/ab_env.sh PINSAGE_WGRAD_PLANES "0 1 0 1" || exit 1
AMD_LOG_LEVEL=3 AMD_LOG_MASK=1 PINSAGE_TEST_CSR_FORK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q -s --timeout 200 --timeout-method thread -k "forked_csr_branch and 2" > $out/fork_api.log 2>&1; echo "forked rc $?"
grep -nE "hipStreamBeginCapture|hipStreamEndCapture|hipStreamWaitEvent|hipEventRecord|hipStreamCreate|hipEventCreate|hipGraphInstantiate" $out/fork_api.log > $out/fork_api_streams.txt; wc -l $out/fork_api_streams.txt; rm -f $out/fork_api.log; tail -30 $out/fork_api_streams.txt
