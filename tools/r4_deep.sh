# Round 4: deep-ring one-workgroup-per-CU tiles (cfg 6: BK 16 x 12 stages, cfg 7: BK 32 x 6) vs cfg 1 / 3
set -o pipefail
out=gpurun_out/r4deep
mkdir -p $out
timeout -k 10 400 python tools/gemm_bench.py --prec 1 --cfgs 1,3,6,7 --sk 0 --reps 30 --pool 100000 --sorted --bias-act --shapes 2600,512,128,1,1,1 10541,512,512,1,1,1 23289,512,128,1,1,1 > $out/q.txt 2>&1 || { tail $out/q.txt; exit 1; }
cat $out/q.txt
timeout -k 10 400 python tools/gemm_bench.py --prec 1 --cfgs 1,3,6,7 --sk 0 --reps 30 --shapes 5709,512,128,1,0,0 8560,512,128,1,0,0 2600,128,512,1,0,0 1536,640,128,1,0,0 > $out/b.txt 2>&1 || { tail $out/b.txt; exit 1; }
cat $out/b.txt
echo ok
