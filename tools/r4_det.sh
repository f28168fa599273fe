# Round 4: two-pass deterministic accumulation, radix pos_csr, parallel split chunks -- tests, bench, traces
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4det
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_micro.py tests/test_gpu_torch_ops.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s.json 2>$out/c4s.err || { tail $out/c4s.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/tc4s -o run -- python3 $R/bench.py --no-cpu-baseline --config c4 --scaling strong --steps 10 > $out/tc4s.json 2> $out/tc4s.err || { tail $out/tc4s.err; exit 1; }
echo ok
