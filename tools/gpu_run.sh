set -o pipefail
out=gpurun_out/r6zg; mkdir -p $out
bash tools/ab_env.sh PINSAGE_FORK_PLAN "0 1 0 1 0 1 0 1" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_aggw.py -x -q --timeout 200 --timeout-method thread > $out/par.log 2>&1 || { tail -30 $out/par.log; exit 1; }
tail -1 $out/par.log
PINSAGE_AGGW32_MIN_ROWS=1000000000 bash tools/ab_env.sh PINSAGE_AGGW_NH "1 0" --config c4 || exit 1
bash tools/ab_env.sh PINSAGE_AGGW32_MIN_ROWS "4096 1000000000 4096 1000000000" --config c4 || exit 1
bash tools/ab_env.sh PINSAGE_AGGW32_MIN_ROWS "4096 1000000000" --config c4 --scaling strong || exit 1
bash tools/ab_env.sh PINSAGE_AGGW32_MIN_ROWS "4096 1000000000" || exit 1
