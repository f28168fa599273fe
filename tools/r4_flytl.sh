# Round 4: kernel trace of the on-the-fly step; GEMM / parity tests after the split-K chunk grid change
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4flytl
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/fly -o run -- python3 $R/bench.py --no-cpu-baseline --sampling fly --steps 10 --warmup 3 > $out/fly.json 2> $out/fly.err || { tail $out/fly.err; exit 1; }
echo ok
