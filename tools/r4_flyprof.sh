# Round 4: host profile of the on-the-fly step, plus graph-timed GEMM microbench
set -o pipefail
out=gpurun_out/r4fly
mkdir -p $out
timeout -k 10 300 python -m cProfile -o $out/fly.prof bench.py --no-cpu-baseline --sampling fly --steps 20 --warmup 3 > $out/fly.json 2> $out/fly.err || { tail $out/fly.err; exit 1; }
tail -1 $out/fly.json | cut -c1-200
timeout -k 10 400 python tools/gemm_bench.py --graph --prec 1 --cfgs 1,3 --sk 0 --reps 40 --bias-act --shapes 64,128,16,1,1 64,128,128,1,1 2600,512,16,1,1 2600,512,128,1,1 2600,512,512,1,1 10541,512,512,1,1 > $out/g.txt 2>&1 || { tail $out/g.txt; exit 1; }
cat $out/g.txt
echo ok
