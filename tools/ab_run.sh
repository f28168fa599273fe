# A/B of PINSAGE_DQ_PROJECT: parity-relevant GPU tests forced on, then bench lines off / on
mkdir -p gpurun_out/ab4
PINSAGE_DQ_PROJECT=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_micro.py tests/test_gpu_dp.py tests/test_gpu_fly.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab4/tests.log 2>&1 || { tail -40 gpurun_out/ab4/tests.log; exit 1; }
tail -1 gpurun_out/ab4/tests.log
for v in 0 1; do
  PINSAGE_DQ_PROJECT=$v timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/ab4/c2_p$v.json 2>/dev/null || exit 1
  PINSAGE_DQ_PROJECT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > gpurun_out/ab4/c4_p$v.json 2>/dev/null || exit 1
  PINSAGE_DQ_PROJECT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > gpurun_out/ab4/c4s_p$v.json 2>/dev/null || exit 1
done
echo ok
