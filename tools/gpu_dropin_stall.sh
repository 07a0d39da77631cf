# drop-in iar (8 MPI ranks on one GPU) repeated with the box's default environment, plus a census of
# the KFD hardware queues each rank process holds while it runs (root cause of the intermittent
# slowdown recorded in round 1)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_stall.jsonl; : > $out
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}" > gpurun_out/dropin_queues.txt
for rep in $(seq 1 ${REPS:-12}); do
  echo "# rep=$rep" >> $out
  timeout -k 5 60 /opt/conda/bin/mpiexec -n ${NR:-8} rootless-coll-mpi-ops_amd/lib/rlo_api_bench iar ${P:-2000} >> $out 2>> gpurun_out/dropin_stall.err &
  bg=$!
  if [ $rep -le 2 ]; then
    sleep 1.5
    echo "--- rep $rep" >> gpurun_out/dropin_queues.txt
    for d in /sys/class/kfd/kfd/proc/*; do
      p=$(basename $d); nq=$(ls $d/queues 2>/dev/null | wc -l)
      echo "pid $p queues $nq $(tr '\0' ' ' < /proc/$p/cmdline 2>/dev/null | cut -c1-60)" >> gpurun_out/dropin_queues.txt
    done
  fi
  wait $bg || exit 1
done
