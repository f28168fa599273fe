# Round 4: GEMM device time under graph replay (no host launch rate)
set -o pipefail
out=gpurun_out/r4ggraph
mkdir -p $out
timeout -k 10 400 python tools/gemm_bench.py --graph --prec 1 --cfgs 1,3 --sk 0 --reps 40 --bias-act --shapes 64,128,16,1,1 64,128,128,1,1 2600,512,16,1,1 2600,512,128,1,1 2600,512,512,1,1 10541,512,512,1,1 > $out/a.txt 2>&1 || { tail $out/a.txt; exit 1; }
cat $out/a.txt
timeout -k 10 400 python tools/gemm_bench.py --graph --prec 1 --cfgs 1,3 --sk 0 --reps 40 --shapes 5709,512,128,1,0,0 2600,128,512,1,0,0 > $out/b.txt 2>&1 || { tail $out/b.txt; exit 1; }
cat $out/b.txt
echo ok
