set -o pipefail
timeout -k 10 300 python tools/gemm_bench.py --graph --reps 20 --cfgs 0,1,2 --sk 0 --shapes 512,512,10544,0,0,1,32 512,512,10544,0,0,1,16 512,512,10544,0,0,1,64 512,512,10544,0,0,0,32 512,512,10544,1,1,0,32 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python tools/gemm_bench.py --graph --reps 20 --cfgs -1,0,1,2,3 --sk 0 --bias-act --shapes 10541,512,512,1,1,1 2>&1 | grep -v amdgpu.ids
