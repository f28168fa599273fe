# Round 4: rep_sum batching, stepper host stats -- tests, benches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4det2
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_micro.py tests/test_gpu_trainer.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
PINSAGE_HOST_TIMING=1 timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2_ht.json 2>$out/c2_ht.err || { tail $out/c2_ht.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s.json 2>$out/c4s.err || { tail $out/c4s.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
echo ok
