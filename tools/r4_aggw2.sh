# Round 4: agg_w32 with loads ahead of stores -- aggw + parity tests, aggw microbench, C2 / C4 / C4 B4096 lines
set -o pipefail
out=gpurun_out/r4aggw2
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_aggw.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s.json 2>$out/c4s.err || { tail $out/c4s.err; exit 1; }
echo ok
