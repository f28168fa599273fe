# A/B of one engine env knob on bench.py: tools/ab_env.sh VAR "A B A B" [bench args]
set -o pipefail
var=$1; vals=$2; shift 2
out=gpurun_out/ab_$var${AB_TAG:+_$AB_TAG}
mkdir -p $out
i=0
for v in $vals; do
  i=$((i+1))
  env $var=$v timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $out/${i}_$v.json 2>$out/${i}_$v.err || { tail $out/${i}_$v.err; exit 1; }
  python tools/bench_summary.py $out/${i}_$v.json | sed "s/^/$var=$v /"
done
