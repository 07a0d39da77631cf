# Diagnostic: drop-in iar stalls with the watchdog on (rootless_ops.cpp watchdog, rlo_client_debug)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/stall.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for i in 1 2 3 4 5; do
  RLO_WATCHDOG=0.5 timeout -k 5 40 $M -n 8 $B iar 2000 > gpurun_out/o.json 2> gpurun_out/wd_$i.txt
  echo "run $i rc=$? $(tail -1 gpurun_out/o.json) watchdog lines $(wc -l < gpurun_out/wd_$i.txt)" >> $out
done
RLO_WATCHDOG=1 timeout -k 5 60 $M -n 8 $B iar 20000 > gpurun_out/o.json 2> gpurun_out/wd_long.txt
echo "long rc=$? $(tail -1 gpurun_out/o.json) watchdog lines $(wc -l < gpurun_out/wd_long.txt)" >> $out
exit 0
