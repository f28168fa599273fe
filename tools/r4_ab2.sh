# Round 4: A/B lines (aggregation + W form; native step host path)
set -o pipefail
out=gpurun_out/r4ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_micro.py tests/test_gpu_fly.py -m gpu -q --timeout 200 --timeout-method thread > $out/tests2.log 2>&1 || { tail -40 $out/tests2.log; exit 1; }
tail -1 $out/tests2.log
for f in 1 0; do
  PINSAGE_AGGW_FORM=$f timeout -k 10 120 python tools/aggw_bench.py --shapes c2l0,c2l1,c4l0,c4sl0 > $out/aggw_bench_f$f.json 2>&1 || { tail $out/aggw_bench_f$f.json; exit 1; }
done
for f in 1 0; do
  PINSAGE_AGGW_FORM=$f timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2_f$f.json 2>$out/c2_f$f.err || { tail $out/c2_f$f.err; exit 1; }
  PINSAGE_AGGW_FORM=$f timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s_f$f.json 2>$out/c4s_f$f.err || { tail $out/c4s_f$f.err; exit 1; }
done
for n in 0 1; do
  PINSAGE_NATIVE_STEP=$n PINSAGE_HOST_TIMING=1 timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2_native$n.json 2>$out/c2_native$n.err || { tail $out/c2_native$n.err; exit 1; }
done
echo ok
