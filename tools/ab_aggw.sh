# A/B of a compile-time variant of the C-ABI (PINSAGE_LIB=libpinsage_hip_b.so):
# its parity tests and bench lines, then the round-end check of the current tree.
set -o pipefail
mkdir -p gpurun_out/ab
B=$PWD/gcn-song-embeddings_amd/libpinsage_hip_b.so
for c in c2 c4; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab/a_$c.json 2>/dev/null || exit 1
  PINSAGE_LIB=$B timeout -k 10 200 python bench.py --no-cpu-baseline --config $c > gpurun_out/ab/b_$c.json 2>/dev/null || exit 1
done
PINSAGE_LIB=$B timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > gpurun_out/ab/b_c4s.json 2>/dev/null || exit 1
PINSAGE_LIB=$B timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/b_tests.log 2>&1 || { tail -30 gpurun_out/ab/b_tests.log; exit 1; }
tail -1 gpurun_out/ab/b_tests.log
echo ab ok
bash tools/round_check.sh
