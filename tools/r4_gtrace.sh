# Round 4: kernel durations of small GEMM launches (rocprofv3 kernel trace of the graph-timed microbench)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4gtrace
mkdir -p $out
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/t1 -o run -- python3 $R/tools/gemm_bench.py --graph --prec 1 --cfgs 3 --sk 0 --reps 40 --bias-act --shapes 64,128,16,1,1 > $out/t1.txt 2>&1 || { tail $out/t1.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/t2 -o run -- python3 $R/tools/gemm_bench.py --graph --prec 1 --cfgs 3 --sk 0 --reps 40 --bias-act --shapes 2600,512,128,1,1 > $out/t2.txt 2>&1 || { tail $out/t2.txt; exit 1; }
cat $out/t1.txt $out/t2.txt | grep prec=
echo ok
