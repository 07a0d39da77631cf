#!/bin/bash
# tests/test_gpu_dropin.py (or FILES) repeated up to REPS times (stop at the first failure) with the drop-in's
# RLO_WATCHDOG state dumps on; logs under gpurun_out/.  REPS=3 bash tools/diag_dropin_pytest.sh
set -o pipefail
mkdir -p gpurun_out
export RLO_WATCHDOG=5
for i in $(seq 1 "${REPS:-3}"); do
    timeout -k 10 300 python -u -m pytest ${FILES:-tests/test_gpu_dropin.py} -x -q --timeout 120 --timeout-method thread \
        > gpurun_out/dp_$i.log 2>&1
    rc=$?
    echo "rep $i: rc=$rc $(tail -1 gpurun_out/dp_$i.log)" | tee -a gpurun_out/dp_summary.txt
    [ $rc -ne 0 ] && exit $rc
done
exit 0
