#!/bin/bash
# A/B: agent acquire between progress iterations (default) vs none (RLO_NO_ACQUIRE, unsafe) on the
# storm / latency / decisions legs, then the fresh-world logged-storm stress.  bash tools/gpu_ab_acq.sh
set -e -o pipefail
mkdir -p gpurun_out
B="python bench.py --no-pmc --no-api --no-bulk --no-cpu-baseline"
timeout -k 10 200 $B > gpurun_out/ab_acq.json 2> gpurun_out/ab_acq.err
RLO_NO_ACQUIRE=1 timeout -k 10 200 $B > gpurun_out/ab_noacq.json 2> gpurun_out/ab_noacq.err
timeout -k 10 200 $B > gpurun_out/ab_acq2.json 2> gpurun_out/ab_acq2.err
timeout -k 10 240 python -u tools/stress_storm_logged.py --fresh --reps 40 > gpurun_out/ss_fresh_acq.log 2>&1
