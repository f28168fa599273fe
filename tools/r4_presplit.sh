# Round 4: Q0 projection with pre-split B planes vs in-register split
set -o pipefail
out=gpurun_out/r4presplit
mkdir -p $out
timeout -k 10 300 python tools/gemm_bench.py --prec 1,2 --cfgs 0,3 --sk 0 --reps 30 --pool 100000 --sorted --bias-act --shapes 10541,512,512,1,1,1 23289,512,128,1,1,1 2600,512,128,1,1,1 > $out/q0.txt 2>&1 || { tail $out/q0.txt; exit 1; }
cat $out/q0.txt
echo ok
