# Round 4: split-bf16 head products + split-K chunk grid: tests, C2 / C4 lines, on-the-fly step trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4head
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_parity.py tests/test_gpu_micro.py tests/test_gpu_configs.py tests/test_gpu_trainer.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/fly -o run -- python3 $R/bench.py --no-cpu-baseline --sampling fly --steps 10 --warmup 3 > $out/fly.json 2> $out/fly.err || { tail $out/fly.err; exit 1; }
echo ok
