# latency program with rank 0's round observations, then the bulk mover sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/lat_quick.py 4 8 64 256 2>&1 | tee gpurun_out/r3_lat_round.txt || exit 1
timeout -k 10 240 python3 tools/bulk_probe.py 16,64,128,0 1,4,64 2>&1 | tee gpurun_out/r3_bulk_probe.txt
