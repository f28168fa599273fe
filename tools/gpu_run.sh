set -o pipefail
out=gpurun_out/r6f; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -30 $out/t1.log; exit 1; }
grep passed $out/t1.log
timeout -k 10 300 python -u tools/wgrad_bench.py > $out/wb.log 2>&1 || { tail -30 $out/wb.log; exit 1; }
cat $out/wb.log
for c in c2 c4; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --config $c > $out/b_${c}.json 2> $out/b_${c}.err || { tail $out/b_${c}.err; exit 1; }
python tools/bench_summary.py $out/b_${c}.json
done
AMD_LOG_LEVEL=3 PINSAGE_CSR_FORK=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread -k "forked and 2" > $out/t3.log 2>&1; echo "forked (look-ahead, HIP log) rc $?"; wc -l $out/t3.log; grep -n "Segmentation\|Fatal" $out/t3.log | head -3; tail -c 60000 $out/t3.log > $out/t3_end.log; rm -f $out/t3.log
