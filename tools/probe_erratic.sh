# Diagnostic: erratic drop-in iar times -- GPU scheduling or host side?  (see tools/probe_erratic.py)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/erratic.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
RLO_TRACE_SETUP=1 timeout -k 5 60 $M -n 4 oracle/_ref/dropin_harness gpurun_out/t2.jsonl tests2 > gpurun_out/tests2_trace.txt 2>&1
echo "tests2 rc=$?" >> $out
for n in /sys/class/kfd/kfd/topology/nodes/*; do echo "node $(basename $n) gpu_id $(cat $n/gpu_id)" >> $out; done
timeout -k 5 90 $M -n 8 $B iar 20000 > gpurun_out/o8.json 2>&1 &
bg=$!
sleep 3
for d in /sys/class/kfd/kfd/proc/*; do
  p=$(basename $d)
  g=$(cat $d/queues/*/gpuid 2>/dev/null | sort | uniq -c | tr '\n' ' ')
  echo "kfd pid $p queues $(ls $d/queues 2>/dev/null | wc -l) gpuids: $g" >> $out
done
wait $bg; echo "iar20000 n=8 rc=$? $(tail -1 gpurun_out/o8.json)" >> $out
for i in 1 2 3 4 5 6; do
  timeout -k 5 90 $M -n 8 $B iar 2000 > gpurun_out/o.json 2>&1 || { echo "rc=$?" >> $out; exit 1; }
  echo "dropin n=8 $(tail -1 gpurun_out/o.json)" >> $out
done
timeout -k 5 120 python3 -u tools/probe_erratic.py 10 >> $out 2>&1 || exit 1
for i in 1 2 3 4; do
  RLO_NO_PUMP=1 timeout -k 5 90 $M -n 8 $B iar 2000 > gpurun_out/o.json 2>&1 || { echo "rc=$?" >> $out; exit 1; }
  echo "dropin nopump n=8 $(tail -1 gpurun_out/o.json)" >> $out
done
