# Round 4: head kernels with all global loads ahead of stores -- probe, tests, C2 / C4 lines
set -o pipefail
out=gpurun_out/r4head2
mkdir -p $out
PINSAGE_LIB=probe/libpinsage_hip.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 2 > $out/hprobe.json 2> $out/hprobe.err || { tail $out/hprobe.err; exit 1; }
grep -a "head_bwd probe" $out/hprobe.err | tail -6
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_micro.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 150 python bench.py --no-cpu-baseline > $out/c2.json 2>$out/c2.err || { tail $out/c2.err; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --config c4 > $out/c4.json 2>$out/c4.err || { tail $out/c4.err; exit 1; }
echo ok
