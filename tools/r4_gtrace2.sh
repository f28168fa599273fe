# Round 4: small-launch kernel durations, cfg 3 (86 KB of code) vs cfg 5 (11 KB)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4gtrace2
mkdir -p $out
export TMPDIR=/tmp
cd /tmp || exit 1
for c in 3 5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/c$c -o run -- python3 $R/tools/gemm_bench.py --graph --prec 1 --cfgs $c --sk 0 --reps 40 --shapes 64,128,32,1,1 > $out/c$c.txt 2>&1 || { tail $out/c$c.txt; exit 1; }
grep prec= $out/c$c.txt
done
echo ok
