#!/bin/bash
# rocprofv3 evidence for one bench configuration (run on the GPU box from the repo root):
#   tools/profile_config.sh NAME [bench.py args...]
# 1. kernel trace + stats of a bench run (its JSON line beside it);
# 2. three --pmc passes, each its own run (FETCH_SIZE; WRITE_SIZE; MFMA busy), per
#    MI355X_MICROARCH.md's HBM / rocprofv3 section.
# Output under gpurun_out/prof_NAME/; summarise with tools/pmc_summary.py,
# tools/pmc_site.py and tools/pmc_mfma.py.
set -o pipefail
name=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/prof_$name
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d "$out/stats" -o run -- \
  python3 "$R/bench.py" --no-cpu-baseline "$@" > "$out/bench.json" 2> "$out/bench.err" || exit 1
echo "[profile] $name stats done"
# the PMC passes re-run the stats run's GEMM choices (the tuner's probes would
# time differently under counters and could pick other kernels)
python3 -c "import json,sys; json.dump(json.load(open(sys.argv[1]))['gemm_choices'], open(sys.argv[2], 'w'))" \
  "$out/bench.json" "$out/gemm_choices.json" || exit 1
export PINSAGE_GEMM_CHOICES="$out/gemm_choices.json"
for pass in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES"; do
  tag=${pass%% *}
  # shellcheck disable=SC2086
  timeout -s KILL 420 rocprofv3 --pmc $pass -f csv -d "$out/pmc_$tag" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 5 --warmup 2 "$@" > "$out/pmc_$tag.json" \
    2> "$out/pmc_$tag.err" || exit 1
  echo "[profile] $name pmc $tag done"
done
