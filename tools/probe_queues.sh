# Diagnostic: how many KFD (hardware) queues each drop-in rank process holds while the
# 8-rank api_bench iar runs on one GPU (root cause of the intermittent drop-in slowdown).
# Usage (GPU box): bash tools/probe_queues.sh [NR] ; env HWQ=n sets GPU_MAX_HW_QUEUES
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/probe_queues.txt
: > $out
echo "GPU_MAX_HW_QUEUES(env)=${GPU_MAX_HW_QUEUES:-unset} HWQ=${HWQ:-}" >> $out
if [ -n "$HWQ" ]; then export GPU_MAX_HW_QUEUES=$HWQ; fi
timeout -k 5 60 /opt/conda/bin/mpiexec -n ${NR:-8} rootless-coll-mpi-ops_amd/lib/rlo_api_bench iar ${P:-20000} > gpurun_out/probe_iar.jsonl 2>&1 &
bg=$!
for t in 1 2 3 4; do
  sleep 1
  echo "--- t=${t}s" >> $out
  for d in /sys/class/kfd/kfd/proc/*; do
    p=$(basename $d)
    nq=$(ls $d/queues 2>/dev/null | wc -l)
    cmd=$(tr '\0' ' ' < /proc/$p/cmdline 2>/dev/null | cut -c1-80)
    echo "pid $p queues $nq cmd $cmd" >> $out
  done
done
wait $bg
echo "iar rc=$?" >> $out
cat gpurun_out/probe_iar.jsonl >> $out
