set -o pipefail
out=gpurun_out/r6n; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "variants_train_alike" > $out/var.log 2>&1 || { tail -30 $out/var.log; exit 1; }
tail -1 $out/var.log
bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 1 3 7 0 1 3 7" || exit 1
bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 7 0 7" --config c4 || exit 1
PINSAGE_KW_SIDE_FORM=1 PINSAGE_KW_SIDE_WG=128 bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 7 3 0 7 3" || exit 1
PINSAGE_TEST_CSR_FORK=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q -s --timeout 200 --timeout-method thread -k "forked" > $out/fork.log 2>&1; echo "forked rc $?"; tail -3 $out/fork.log
