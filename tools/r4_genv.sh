# Round 4: HIP graph runtime settings A/B on the C2 step (graph launch host time, ms/step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4genv
mkdir -p $out
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 150 python bench.py --no-cpu-baseline > $out/$n.json 2>$out/$n.err || { tail $out/$n.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_ms_per_step']; print(sys.argv[2], round(d['ms_per_step'],4), round(h['native_call'],4), round(h['graph_launch'],4), round(h['train_batch_enqueue_excl_ring_wait'],4))" $out/$n.json $n
}
run base X=1 && run pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && run pc1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 && run fq1 DEBUG_HIP_FORCE_GRAPH_QUEUES=1 && run fq4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 && run bs64 DEBUG_HIP_GRAPH_BATCH_SIZE=64 && run bs8 DEBUG_HIP_GRAPH_BATCH_SIZE=8 && echo ok
