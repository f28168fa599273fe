# Round 4: warp-specialised GEMM (cfg 5), canonical CSR via bitmap ranking, reproducibility; C2 / C4 lines
set -o pipefail
out=gpurun_out/r4ab3
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q --timeout 200 --timeout-method thread -k "warp_specialised or layouts" > $out/tests_gemm.log 2>&1 || { tail -40 $out/tests_gemm.log; exit 1; }
tail -1 $out/tests_gemm.log
timeout -k 10 200 python tools/gemm_bench.py --prec 1 --cfgs 3,5 --sk 0 --reps 30 --pool 100000 --sorted --bias-act --shapes 10541,512,512,1,1,1 2600,512,128,1,1,1 23190,512,128,1,1,1 151820,512,128,1,1,1 > $out/gemm_bench.txt 2>&1 || { tail $out/gemm_bench.txt; exit 1; }
cat $out/gemm_bench.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_micro.py tests/test_gpu_configs.py -m gpu -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
PINSAGE_CSR_CANON=0 timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2_nocanon.json 2>$out/c2_nocanon.err || { tail $out/c2_nocanon.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s.json 2>$out/c4s.err || { tail $out/c4s.err; exit 1; }
echo ok
