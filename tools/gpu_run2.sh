set -o pipefail
out=gpurun_out/r5mz; mkdir -p $out
for v in "base" "PINSAGE_FUSED_NEXT_Q=0" "PINSAGE_HEAD_IN_AGGW=0" "PINSAGE_FUSED_NEXT_Q=0 PINSAGE_HEAD_IN_AGGW=0" "PINSAGE_FUSED_AGGW=0"; do
for cfg in "2 10 7" "3 50 16"; do
env TAG="$v" $([ "$v" = base ] || echo $v) timeout -k 10 120 python tools/dbg/micro_z.py $cfg 2>&1 | grep -v amdgpu.ids | tail -n 2
done; done
