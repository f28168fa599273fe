mkdir -p gpurun_out/ab2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fly.py tests/test_gpu_baselines.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/tests_main.log 2>&1 || { tail -30 gpurun_out/ab2/tests_main.log; exit 1; }
tail -1 gpurun_out/ab2/tests_main.log
PINSAGE_LIB=$PWD/gcn-song-embeddings_amd/variants/dq8/libpinsage_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_micro.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/tests_dq8.log 2>&1 || { tail -30 gpurun_out/ab2/tests_dq8.log; exit 1; }
tail -1 gpurun_out/ab2/tests_dq8.log
for v in 16 8 12; do
  L=""; [ $v != 16 ] && L=$PWD/gcn-song-embeddings_amd/variants/dq$v/libpinsage_hip.so
  PINSAGE_LIB=$L timeout -k 10 150 python bench.py --no-cpu-baseline > gpurun_out/ab2/c2_dq$v.json 2>/dev/null || exit 1
  PINSAGE_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > gpurun_out/ab2/c4s_dq$v.json 2>/dev/null || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --sampling fly > gpurun_out/ab2/c2_fly.json 2>/dev/null || exit 1
echo ok
