set -o pipefail
out=gpurun_out/r6c; mkdir -p $out
timeout -k 10 120 ./tools/dbg/capture_fork_probe > $out/capture_probe.log 2>&1; echo "probe rc $?"; grep -E "end|replay|CHILD|child|eager" $out/capture_probe.log | grep reuse
timeout -k 10 600 python -u -m pytest tests/test_gpu_wgrad.py tests/test_gpu_fly_fused.py tests/test_gpu_trainer.py -x -v --timeout 200 --timeout-method thread -k "wgrad or refuses or forked" > $out/t1.log 2>&1 || { tail -60 $out/t1.log; exit 1; }
grep -cE "PASSED" $out/t1.log; grep -E "FAIL" $out/t1.log | head
for rep in 1 2; do for v in "0 0" "1 0" "1 1"; do set -- $v; for c in c2 c4; do
PINSAGE_WGRAD_KW=$1 PINSAGE_DQ_CHUNK_ROWS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --config $c > $out/b_${c}_$1$2_$rep.json 2> $out/b_${c}_$1$2_$rep.err || { tail $out/b_${c}_$1$2_$rep.err; exit 1; }
echo "kw=$1 cr=$2 $(python tools/bench_summary.py $out/b_${c}_$1$2_$rep.json)"
done; done; done
bash tools/prof_timeline.sh $out c2 || exit 1
