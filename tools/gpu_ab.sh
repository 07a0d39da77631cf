#!/bin/bash
# A/B: eager vs lazy counter publish (RLO_LAZY_PUB) on the storm / latency / decisions legs and
# the per-phase latency anatomy.  Run on the GPU box: bash tools/gpu_ab.sh
set -e -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-pmc --no-api --no-bulk --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/ab_eager.json 2> gpurun_out/ab_eager.err
RLO_LAZY_PUB=1 timeout -k 10 200 $B > gpurun_out/ab_lazy.json 2> gpurun_out/ab_lazy.err
timeout -k 10 150 python tools/lat_anatomy.py --n 8 > gpurun_out/ab_la8.log 2>&1
timeout -k 10 150 python tools/lat_anatomy.py --n 256 > gpurun_out/ab_la256.log 2>&1
