set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/diag_bulk.log
for rep in $(seq 1 ${REPS:-1}); do
for s in ${STEPS:-1 2 3 4 5}; do
  echo "=== rep $rep step $s" >> gpurun_out/diag_bulk.log
  timeout -k 10 120 python -u tools/diag_bulk.py $s >> gpurun_out/diag_bulk.log 2>&1 || exit 1
done
done
