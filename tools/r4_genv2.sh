# Round 4: HIP graph queue count A/B on C2 and C4 B4096
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r4genv2
mkdir -p $out
run() {  # name, cfg args, env...
  local n=$1; local a=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline $a > $out/$n.json 2>$out/$n.err || { tail $out/$n.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); h=d['host_ms_per_step']; print(sys.argv[2], round(d['ms_per_step'],4), round(h['native_call'],4), round(h['graph_launch'],4), round(h['train_batch_enqueue_excl_ring_wait'],4))" $out/$n.json $n
}
run fq2 "" DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run fq3 "" DEBUG_HIP_FORCE_GRAPH_QUEUES=3 && run base "" X=1 && run fq2b "" DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run c4s_base "--config c4 --scaling strong" X=1 && run c4s_fq2 "--config c4 --scaling strong" DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && run c4_base "--config c4" X=1 && run c4_fq2 "--config c4" DEBUG_HIP_FORCE_GRAPH_QUEUES=2 && echo ok
