set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/probe/fanout_probe 2>&1 | tee gpurun_out/r3_fanout_probe.txt
