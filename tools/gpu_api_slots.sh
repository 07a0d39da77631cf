# drop-in iar at several ring depths (RLO_RING_SLOTS), 8 ranks, repeated (looks for intermittent stalls)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/api_slots.jsonl; : > $out
for s in ${SLOTS:-512 2048}; do
  for rep in 1 2 3 4 5 6; do
    echo "# slots=$s iar rep=$rep" >> $out
    RLO_RING_SLOTS=$s timeout -k 5 60 /opt/conda/bin/mpiexec -n 8 rootless-coll-mpi-ops_amd/lib/rlo_api_bench iar 2000 >> $out 2>> gpurun_out/api_slots.err || exit 1
  done
done
