# Diagnostic: does the drop-in's 8-rank iar slow down when more processes than the hardware
# scheduler maps at once hold GPU queues?  base (8 ranks) / 8 ranks beside one idle torch process /
# 9 and 12 ranks.  Usage (GPU box): bash tools/probe_oversub.sh
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/probe_oversub.txt
: > $out
run_iar() {  # label nranks reps
  for i in $(seq ${3:-4}); do
    s=$(date +%s.%N)
    timeout -k 5 60 /opt/conda/bin/mpiexec -n $2 rootless-coll-mpi-ops_amd/lib/rlo_api_bench iar 2000 > gpurun_out/o.json 2>&1
    rc=$?
    e=$(date +%s.%N)
    echo "$1 rc=$rc wall=$(python3 -c "print(round($e-$s,2))") $(tail -1 gpurun_out/o.json)" >> $out
    [ $rc -eq 0 ] || return 1
  done
}
run_iar base8 8 4 || exit 1
rm -f gpurun_out/dummy_ready
timeout -k 5 120 python3 -c "
import torch, time
x = torch.ones(1, device='cuda'); torch.cuda.synchronize()
s = torch.cuda.Stream(); y = x + 1; torch.cuda.synchronize()
open('gpurun_out/dummy_ready', 'w').close(); time.sleep(90)" &
dummy=$!
for i in $(seq 90); do [ -f gpurun_out/dummy_ready ] && break; sleep 1; done
for d in /sys/class/kfd/kfd/proc/*; do echo "kfd pid $(basename $d) queues $(ls $d/queues 2>/dev/null | wc -l)" >> $out; done
run_iar idle_torch_beside 8 4
rc=$?
kill $dummy 2>/dev/null; wait $dummy 2>/dev/null
[ $rc -eq 0 ] || exit 1
run_iar n9 9 3 && run_iar n12 12 3
