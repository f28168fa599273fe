# Round 4: the fragment-form aggregation + W kernel against the LDS-tile form
# (PINSAGE_AGGW_FORM=0) -- its parity tests, the microbenchmark and in-step bench lines.
set -o pipefail
out=gpurun_out/r4ab
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_aggw.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > $out/test_aggw.log 2>&1 || { tail -30 $out/test_aggw.log; exit 1; }
tail -1 $out/test_aggw.log
for f in 1 0; do
  PINSAGE_AGGW_FORM=$f timeout -k 10 120 python tools/aggw_bench.py --shapes c2l0,c2l1,c4l0,c4sl0 > $out/aggw_bench_f$f.json 2>&1 || { tail $out/aggw_bench_f$f.json; exit 1; }
done
for f in 1 0 1 0; do
  PINSAGE_AGGW_FORM=$f timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2_f$f.json 2>$out/c2_f$f.err || { tail $out/c2_f$f.err; exit 1; }
  PINSAGE_AGGW_FORM=$f timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 --scaling strong > $out/c4s_f$f.json 2>$out/c4s_f$f.err || { tail $out/c4s_f$f.err; exit 1; }
done
echo ok
