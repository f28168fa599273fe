# Round 4: GEMM without the inlined stream-K copy (cfg 0/3/4): tests, small-launch latency, C2/C4 lines
set -o pipefail
out=gpurun_out/r4sk
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests_gemm.log 2>&1 || { tail -30 $out/tests_gemm.log; exit 1; }
tail -1 $out/tests_gemm.log
timeout -k 10 300 python tools/gemm_bench.py --graph --prec 1 --cfgs 1,3 --sk 0 --reps 40 --bias-act --shapes 64,128,32,1,1 2600,512,128,1,1 10541,512,512,1,1 > $out/g.txt 2>&1 || { tail $out/g.txt; exit 1; }
cat $out/g.txt
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
echo ok
