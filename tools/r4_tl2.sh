# Round 4: kernel traces of the C2 and C4 (B512) steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4tl2
mkdir -p $out
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/c4 -o run -- python3 $R/bench.py --no-cpu-baseline --config c4 --steps 10 > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/c2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $out/c2.json 2> $out/c2.err || { tail $out/c2.err; exit 1; }
echo ok
