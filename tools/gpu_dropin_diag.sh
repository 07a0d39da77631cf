# drop-in erratic n>=8: per-rank loop gaps / round latencies / context switches, proxy gaps, cgroup throttling
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_diag.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
grep -E "Cpus_allowed_list" /proc/self/status >> $out
cg=/sys/fs/cgroup/cpu.stat
for n in 8; do
  for rep in 1 2 3 4 5 6; do
    echo "== n=$n rep=$rep load $(cut -d' ' -f1-3 /proc/loadavg) throttled_before $(grep throttled_usec $cg 2>/dev/null)" >> $out
    API_DIAG=1 RLO_PROXY_DIAG=1 timeout -k 5 90 $M -n $n $B iardj 2000 >> $out 2>&1 || { echo "rc=$?" >> $out; exit 1; }
    echo "   throttled_after $(grep throttled_usec $cg 2>/dev/null)" >> $out
  done
done
cat $out
