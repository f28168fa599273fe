set -o pipefail
out=gpurun_out/r5ai; R=$(pwd); mkdir -p $out
for rep in 1 2 3; do for v in start fwd graph late; do
PINSAGE_FRONTIER_AHEAD=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $out/b_${v}_$rep.json 2> $out/b_${v}_$rep.err || { tail $out/b_${v}_$rep.err; exit 1; }
done; done
python - <<'PY'
import json, statistics as st
for v in ["start","fwd","graph","late"]:
    xs=[json.load(open(f"gpurun_out/r5ai/b_{v}_{r}.json"))["ms_per_step"] for r in (1,2,3)]
    print("ahead", v, "median %.4f" % st.median(xs), ["%.4f" % x for x in xs])
PY
