#!/bin/bash
# The reference's testcases.c wrappers through the drop-in at 8 ranks ("tests_safe"), repeated up
# to REPS times, stopping at the first failure; RLO_WATCHDOG dumps engine state when a rank stops
# seeing events.  Output under gpurun_out/.  REPS=5 bash tools/diag_dropin8.sh
set -o pipefail
mkdir -p gpurun_out
cd gpurun_out
for i in $(seq 1 "${REPS:-5}"); do
    t0=$(date +%s.%N)
    RLO_WATCHDOG=5 RLO_TRACE=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n 8 ../oracle/_ref/dropin_harness d8_$i.jsonl tests_safe > d8_$i.log 2>&1
    rc=$?
    echo "rep $i: rc=$rc seconds=$(python3 -c "import time; print(round(time.time() - $t0, 1))")" | tee -a d8_summary.txt
    [ $rc -ne 0 ] && exit $rc
done
exit 0
