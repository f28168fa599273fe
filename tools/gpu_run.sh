set -o pipefail
out=gpurun_out/r5h; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fly_fused.py > $out/t.log 2>&1; rc=$?
tail -30 $out/t.log
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --sampling fly > $out/bench_c2_fly.json 2> $out/bench_c2_fly.err || { tail $out/bench_c2_fly.err; exit 1; }
python tools/bench_summary.py $out/bench_c2_fly.json
