set -o pipefail
out=gpurun_out/r6p; mkdir -p $out
timeout -k 10 200 python -u tools/wgrad_bench.py > $out/wb.log 2>&1 || { tail -30 $out/wb.log; exit 1; }
grep -v amdgpu.ids $out/wb.log
PINSAGE_KW_SIDE_FORM=1 PINSAGE_KW_SIDE_WG=128 bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 3 0 3" || exit 1
bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 3 0 3" || exit 1
bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 3 0 3" --config c4 || exit 1
PINSAGE_TEST_CSR_FORK=1 PINSAGE_SEGV_BT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q -s --timeout 200 --timeout-method thread -k "forked_csr_branch and 2" > $out/fork.log 2>&1; echo "forked rc $?"; grep -A45 "segv_bt" $out/fork.log | head -60
