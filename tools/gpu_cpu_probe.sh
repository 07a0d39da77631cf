# Diagnostic: the box's CPU budget (cgroup quota / throttling) around drop-in iar runs, and the
# setup trace of the two-engines-per-process case (tests2).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cpu_probe.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
echo "nproc $(nproc)" >> $out
cat /sys/fs/cgroup/cpu.max >> $out 2>&1
grep -E "nr_periods|nr_throttled|throttled_usec" /sys/fs/cgroup/cpu.stat >> $out 2>&1
for n in 4 8 12 16; do
  for pump in on off; do
    if [ $pump = off ]; then export RLO_NO_PUMP=1; else unset RLO_NO_PUMP; fi
    t0=$(grep throttled_usec /sys/fs/cgroup/cpu.stat | awk '{print $2}')
    timeout -k 5 90 $M -n $n $B iar 2000 > gpurun_out/o.json 2>&1 || { echo "n=$n rc=$?" >> $out; exit 1; }
    t1=$(grep throttled_usec /sys/fs/cgroup/cpu.stat | awk '{print $2}')
    echo "n=$n pump=$pump throttled_ms=$(( (t1 - t0) / 1000 )) $(tail -1 gpurun_out/o.json)" >> $out
  done
done
unset RLO_NO_PUMP
RLO_TRACE_SETUP=1 timeout -k 5 40 $M -n 4 oracle/_ref/dropin_harness gpurun_out/t2.jsonl tests2 > gpurun_out/tests2_trace.txt 2>&1
echo "tests2 rc=$?" >> $out
