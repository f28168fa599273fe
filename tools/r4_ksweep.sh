# Round 4: GEMM fixed cost and per-k-step cost (K sweep at one tile round)
set -o pipefail
out=gpurun_out/r4ksweep
mkdir -p $out
timeout -k 10 300 python tools/gemm_bench.py --prec 1 --cfgs 1,3 --sk 0 --reps 50 --bias-act --shapes 64,128,16,1,1 64,128,128,1,1 2600,512,16,1,1 2600,512,32,1,1 2600,512,64,1,1 2600,512,128,1,1 2600,512,256,1,1 2600,512,512,1,1 2600,512,1024,1,1 > $out/k.txt 2>&1 || { tail $out/k.txt; exit 1; }
cat $out/k.txt
echo ok
