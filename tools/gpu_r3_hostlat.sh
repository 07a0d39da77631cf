# host-service latency anatomy: host wall (post -> last pickup) vs the device's origination -> last pickup record
set -o pipefail
mkdir -p gpurun_out
for n in 4 8; do timeout -k 10 120 python3 tools/host_latency.py --n $n --rounds 400 || exit 1; done 2>&1 | tee gpurun_out/r3_host_latency.txt
