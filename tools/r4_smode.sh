# Round 4: backward stream modes A/B (ms/step, host launch)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4smode
mkdir -p $out
run() {  # name, cfg args, env...
  local n=$1; local a=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline $a > $out/$n.json 2>$out/$n.err || { tail $out/$n.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_ms_per_step']; print(sys.argv[2], round(d['ms_per_step'],4), round(h['native_call'],4), round(h['graph_launch'],4), round(h['train_batch_enqueue_excl_ring_wait'],4))" $out/$n.json $n
}
for m in 0 2 4 0 2 4; do run c2_m$m "" PINSAGE_BWD_STREAMS=$m || exit 1; done
for m in 0 2 4; do run c4_m$m "--config c4" PINSAGE_BWD_STREAMS=$m || exit 1; done
echo ok
