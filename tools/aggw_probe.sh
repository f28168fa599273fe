# Phase probe of agg_w32 (timing only, results wrong; build the probes first
# with tools/aggw_probe_build.py): p1 = projection loop
# removed (gather + epilogue), p2 = gather removed (projection + epilogue).
set -o pipefail
mkdir -p gpurun_out/probe
L=$PWD/gcn-song-embeddings_amd
for c in c2 c4s; do
  for v in a p1 p2; do
    lib=$L/libpinsage_hip.so; [ $v != a ] && lib=$L/libpinsage_hip_$v.so
    if [ $c = c4s ]; then extra="--config c4 --scaling strong"; else extra="--config c2"; fi
    PINSAGE_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline $extra --steps 20 > gpurun_out/probe/${v}_$c.json 2> gpurun_out/probe/${v}_$c.err || { tail -5 gpurun_out/probe/${v}_$c.err; exit 1; }
  done
done
echo probe ok
