set -o pipefail
out=gpurun_out/r5ah; R=$(pwd); mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gputest.log 2>&1 || { tail -n 30 $out/gputest.log; exit 1; }
tail -n 1 $out/gputest.log
for rep in 1 2 3 4; do
timeout -k 10 200 python bench.py --no-cpu-baseline > $out/b_$rep.json 2> $out/b_$rep.err || { tail $out/b_$rep.err; exit 1; }
python - $out/b_$rep.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); k=d["kernels"]
print("bench", round(d["value"]), round(d["ms_per_step"],4), "frontier", round(k["fwd.frontier"]["avg_ms"]*1e3,1), "l0", round(k["bwd.layer.l0"]["avg_ms"]*1e3,1), "graph_launch", round(d["host_ms_per_step"]["graph_launch"],3), flush=True)
PY
done
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2> $out/c4.err || { tail $out/c4.err; exit 1; }
python - $out/c4.json <<'PY'
import json,sys
d=json.load(open(sys.argv[1])); k=d["kernels"]
print("c4", round(d["value"]), round(d["ms_per_step"],4), "frontier", round(k["fwd.frontier"]["avg_ms"]*1e3,1), flush=True)
PY
