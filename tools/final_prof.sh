# The default bench line on the final tree, then a rocprofv3 kernel-stats pass of
# the same C2 command (its summary is copied to profiles/).
set -o pipefail
R=$PWD
mkdir -p gpurun_out/s4
timeout -k 10 240 python bench.py > gpurun_out/s4/bench_c2.json 2> gpurun_out/s4/bench_c2.err || { tail -20 gpurun_out/s4/bench_c2.err; exit 1; }
cat gpurun_out/s4/bench_c2.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/s4/prof -o c2 -- python3 $R/bench.py --no-cpu-baseline --steps 20 > gpurun_out/s4/prof_c2_bench.json 2> gpurun_out/s4/prof.err || { tail -20 gpurun_out/s4/prof.err; exit 1; }
find gpurun_out/s4/prof -name "*stats*" | head
echo prof ok
