# the drop-in's consensus loop with and without the proposal pool, 8 rank processes on one GPU
set -o pipefail
mkdir -p gpurun_out
for spec in "1 iardj 2000" "16 iardj 2000" "16 iarpool 8000" "4 iarpool 8000"; do
  set -- $spec
  echo "== RLO_PROPOSAL_POOL=$1 $2 $3"
  RLO_PROPOSAL_POOL=$1 timeout -k 5 120 /opt/conda/bin/mpiexec -n 8 rootless-coll-mpi-ops_amd/lib/rlo_api_bench $2 $3 > gpurun_out/api_$1_$2.log 2>&1; rc=$?
  grep mode gpurun_out/api_$1_$2.log || tail -15 gpurun_out/api_$1_$2.log
  [ $rc -eq 0 ] || { echo "rc=$rc"; exit 1; }
done
