set -o pipefail
out=gpurun_out/r5g; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -rf > $out/gputest.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error" $out/gputest.log | tail -15
[ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > $out/bench_c2.json 2> $out/bench_c2.err || { tail $out/bench_c2.err; exit 1; }
python tools/bench_summary.py $out/bench_c2.json
timeout -k 10 300 python bench.py --no-cpu-baseline --config c3 > $out/bench_c3.json 2> $out/bench_c3.err || { tail $out/bench_c3.err; exit 1; }
python tools/bench_summary.py $out/bench_c3.json
timeout -k 10 600 python bench.py --no-cpu-baseline --config c5 > $out/bench_c5.json 2> $out/bench_c5.err || { tail $out/bench_c5.err; exit 1; }
python tools/bench_summary.py $out/bench_c5.json
