set -o pipefail
out=gpurun_out/r6x; mkdir -p $out
bash tools/ab_env.sh DEBUG_HIP_FORCE_GRAPH_QUEUES "4 2 3 4 2 3" || exit 1
PINSAGE_SEGV_BT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -v -s --timeout 200 --timeout-method thread -k "forked_csr_branch" > $out/fork.log 2>&1; rc=$?; echo "forked rc $rc"; grep -E "PASS|FAIL|passed|failed|segv_bt\]" $out/fork.log | head
