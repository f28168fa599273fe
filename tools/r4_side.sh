# Round 4: grid cap of the backward's side-stream weight gradients (interference with the chain)
set -o pipefail
out=gpurun_out/r4side
mkdir -p $out
run() {  # name, cfg args, env...
  local n=$1; local a=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline $a > $out/$n.json 2>$out/$n.err || { tail $out/$n.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],4))" $out/$n.json $n
}
for g in 0 256 128 0 256 128; do run c2_g$g "" PINSAGE_SIDE_GRID=$g || exit 1; done
for g in 0 256 128; do run c4_g$g "--config c4" PINSAGE_SIDE_GRID=$g || exit 1; done
echo ok
