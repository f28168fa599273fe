# Kernel trace of bench.py runs (graph replays) for step timelines:
#   tools/prof_timeline.sh OUTDIR [configs...]   (run on the GPU box from the repo root)
set -o pipefail
out=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$out"
export TMPDIR=/tmp
for c in "$@"; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$R/$out/tr_$c" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --config $c --steps 30 > "$R/$out/b_$c.json" 2> "$R/$out/b_$c.err") || exit 1
  f=$(ls "$R/$out"/tr_$c/*/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -z "$f" ] && f=$(find "$R/$out/tr_$c" -name "*kernel_trace.csv" | head -1)
  python3 "$R/tools/timeline.py" "$f" --step 20 > "$R/$out/timeline_$c.txt" || exit 1
  echo "[prof] $c done"; tail -3 "$R/$out/timeline_$c.txt"
done
