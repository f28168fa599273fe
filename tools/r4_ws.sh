# Round 4: warp-specialised GEMM variants vs cfg 3 on the projection shapes
set -o pipefail
out=gpurun_out/r4ws
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q --timeout 200 --timeout-method thread -k "warp_specialised" > $out/tests_gemm.log 2>&1 || { tail -40 $out/tests_gemm.log; exit 1; }
tail -1 $out/tests_gemm.log
for v in 0 1 2; do
  PINSAGE_WS_VARIANT=$v timeout -k 10 200 python tools/gemm_bench.py --prec 1 --cfgs 3,5 --sk 0 --reps 30 --pool 100000 --sorted --bias-act --shapes 10541,512,512,1,1,1 2600,512,128,1,1,1 23190,512,128,1,1,1 > $out/gemm_bench_v$v.txt 2>&1 || { tail $out/gemm_bench_v$v.txt; exit 1; }
  cat $out/gemm_bench_v$v.txt
done
PINSAGE_WS_VARIANT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -m gpu -q --timeout 200 --timeout-method thread -k "warp_specialised" > $out/tests_gemm1.log 2>&1 || { tail -40 $out/tests_gemm1.log; exit 1; }
tail -1 $out/tests_gemm1.log
echo ok
