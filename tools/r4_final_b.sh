# Round 4 end: rocprofv3 kernel stats + PMC passes (FETCH_SIZE / WRITE_SIZE / MFMA busy) of the C2 and C4 lines
set -o pipefail
timeout -k 10 560 bash tools/profile_config.sh c2 && timeout -k 10 560 bash tools/profile_config.sh c4 --config c4 && echo ok
