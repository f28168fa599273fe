# Round end on one MI355X: GPU suite, smoke(), the default bench line (C2 + CPU baseline), the C4 / C4-B4096 / fly lines, then rocprofv3 kernel stats + PMC passes of C2 and C4 (tools/profile_config.sh; summarise with tools/pmc_sites_all.py)
set -o pipefail
out=gpurun_out/round_end
mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gputest.log 2>&1 || { tail -40 $out/gputest.log; exit 1; }
tail -1 $out/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 240 python bench.py > $out/bench_c2.json 2> $out/bench_c2.err || { tail $out/bench_c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/bench_c4.json 2> $out/bench_c4.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/bench_c4s.json 2> $out/bench_c4s.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --sampling fly > $out/bench_c2_fly.json 2> $out/bench_c2_fly.err || exit 1
echo lines ok

timeout -k 10 560 bash tools/profile_config.sh c2 && timeout -k 10 560 bash tools/profile_config.sh c4 --config c4 && echo ok
