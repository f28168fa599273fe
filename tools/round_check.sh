# Round-end check of the current tree on one MI355X: the GPU suite, smoke(), the
# default bench line (C2 + CPU baseline), the fly / C4 / C4-B4096 lines.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/gputest.log 2>&1 || { tail -40 gpurun_out/final/gputest.log; exit 1; }
tail -1 gpurun_out/final/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 240 python bench.py > gpurun_out/final/bench_c2.json 2> gpurun_out/final/bench_c2.err || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --sampling fly > gpurun_out/final/bench_c2_fly.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > gpurun_out/final/bench_c4.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > gpurun_out/final/bench_c4s.json 2>/dev/null || exit 1
echo ok
