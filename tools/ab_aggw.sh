# A/B/C of compile-time variants of the C-ABI (PINSAGE_LIB=libpinsage_hip_{b,c}.so):
# bench lines interleaved with the current build, then each variant's parity tests.
set -o pipefail
mkdir -p gpurun_out/ab2
L=$PWD/gcn-song-embeddings_amd
for c in c2 c4; do
  for v in a b c; do
    lib=$L/libpinsage_hip.so; [ $v != a ] && lib=$L/libpinsage_hip_$v.so
    PINSAGE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab2/${v}_$c.json 2>/dev/null || exit 1
  done
done
for v in b c; do
  PINSAGE_LIB=$L/libpinsage_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab2/${v}_tests.log 2>&1 || { tail -30 gpurun_out/ab2/${v}_tests.log; exit 1; }
  tail -1 gpurun_out/ab2/${v}_tests.log
done
for v in a b c; do
  lib=$L/libpinsage_hip.so; [ $v != a ] && lib=$L/libpinsage_hip_$v.so
  PINSAGE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > gpurun_out/ab2/${v}_c4s.json 2>/dev/null || exit 1
done
echo ab ok
