# A/B of a compile-time variant of the C-ABI (PINSAGE_LIB=libpinsage_hip_f.so):
# bench lines interleaved with the current build, then the variant's parity tests.
set -o pipefail
mkdir -p gpurun_out/ab3
L=$PWD/gcn-song-embeddings_amd
PINSAGE_LIB=$L/libpinsage_hip_f.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab3/f_tests.log 2>&1 || { tail -30 gpurun_out/ab3/f_tests.log; exit 1; }
tail -1 gpurun_out/ab3/f_tests.log
for c in c2 c4 c4s; do
  if [ $c = c4s ]; then extra="--config c4 --scaling strong"; else extra="--config $c"; fi
  for v in a f a2 f2; do
    lib=$L/libpinsage_hip.so; case $v in f*) lib=$L/libpinsage_hip_f.so;; esac
    PINSAGE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $extra > gpurun_out/ab3/${v}_$c.json 2>/dev/null || exit 1
  done
done
echo ab ok
