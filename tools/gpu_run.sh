set -o pipefail
out=gpurun_out/r5w; R=$(pwd); mkdir -p $out
for rep in 1 2 3 4 5 6 7 8; do for v in 0 1 2; do
PINSAGE_FEATURE_TABLE=$((v>0)) PINSAGE_WTAB_Q=$((v==1)) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $out/b${v}_$rep.json 2> $out/b${v}_$rep.err || { tail $out/b${v}_$rep.err; exit 1; }
done; done
python - <<'PY'
import json, statistics as st
for v in range(3):
    xs=[json.load(open(f"gpurun_out/r5w/b{v}_{r}.json"))["ms_per_step"] for r in range(1,9)]
    q=[json.load(open(f"gpurun_out/r5w/b{v}_{r}.json"))["kernels"]["fwd.q_gemm.l0"]["avg_ms"]*1e3 for r in range(1,9)]
    print("variant", v, "median %.4f mean %.4f min %.4f" % (st.median(xs), st.mean(xs), min(xs)), "q0 %.1f" % st.mean(q))
PY
