# Round 4: C2 kernel trace after the head staging / dq pipelining changes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4tl4
mkdir -p $out
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/c2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $out/c2.json 2> $out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/c4s -o run -- python3 $R/bench.py --no-cpu-baseline --config c4 --scaling strong --steps 10 > $out/c4s.json 2> $out/c4s.err || { tail $out/c4s.err; exit 1; }
echo ok
