set -o pipefail
out=gpurun_out/r5al; R=$(pwd); mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trainer.py -x -q --timeout 300 --timeout-method thread > $out/t.log 2>&1 || { tail -n 30 $out/t.log; exit 1; }
tail -n 1 $out/t.log
for rep in 1 2 3 4; do for v in 0 1; do for c in c2 c4; do
PINSAGE_WG2=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --config $c > $out/b_${c}_${v}_$rep.json 2> $out/b_${c}_${v}_$rep.err || { tail $out/b_${c}_${v}_$rep.err; exit 1; }
done; done; done
python - <<'PY'
import json, statistics as st
for c in ("c2","c4"):
  for v in (0,1):
    ds=[json.load(open(f"gpurun_out/r5al/b_{c}_{v}_{r}.json")) for r in (1,2,3,4)]
    print("wg2", c, v, "median %.4f" % st.median([d["ms_per_step"] for d in ds]), ["%.4f" % d["ms_per_step"] for d in ds])
PY
