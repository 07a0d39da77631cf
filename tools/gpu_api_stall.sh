# drop-in iar repeated under RLO_WATCHDOG until the first slow run (diagnostics for the intermittent stall)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/api_stall.jsonl; : > $out; : > gpurun_out/api_stall.err
for rep in $(seq 1 ${REPS:-16}); do
  echo "# rep=$rep" >> $out
  echo "# rep=$rep" >> gpurun_out/api_stall.err
  RLO_WATCHDOG=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n ${NR:-8} rootless-coll-mpi-ops_amd/lib/rlo_api_bench iar 2000 >> $out 2>> gpurun_out/api_stall.err || exit 1
  if grep -q "rlo watchdog" gpurun_out/api_stall.err; then break; fi
done
