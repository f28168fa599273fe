# Round 4: short-K GEMM shapes (C4 / C2 backward and C4 Q0) under every tile config and both product forms
set -o pipefail
out=gpurun_out/r4shortk
mkdir -p $out
timeout -k 10 300 python tools/gemm_bench.py --prec 0,1 --cfgs 0,1,2,3 --sk 0 --reps 30 --shapes 8560,512,128,1,0,0 5709,512,128,1,0,0 5709,1024,128,1,0,0 > $out/dcat.txt 2>&1 || { tail $out/dcat.txt; exit 1; }
cat $out/dcat.txt
timeout -k 10 300 python tools/gemm_bench.py --prec 0,1 --cfgs 0,1,2,3 --sk 0 --reps 30 --pool 8000000 --sorted --bias-act --shapes 23289,512,128,1,1,1 10541,512,512,1,1,1 > $out/q0.txt 2>&1 || { tail $out/q0.txt; exit 1; }
cat $out/q0.txt
echo ok
