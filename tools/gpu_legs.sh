# the drop-in's legs: api_bench lat / iar under RLO_TRACE_DIR, split by tools/dropin_legs.py
set -o pipefail
tag=${1:-legs}
O=gpurun_out/${RLO_OUT:-r6}/$tag
mkdir -p $O
B=${BENCH:-rootless-coll-mpi-ops_amd/lib/rlo_api_bench}
export RLO_NUMA_BIND=all
for n in ${NS:-4 8}; do
  for leg in "lat 500 64" "iar 2000"; do
    d=$O/n${n}_${leg%% *}; mkdir -p $d
    RLO_TRACE_DIR=$d timeout -k 5 120 /opt/conda/bin/mpiexec -n $n $B $leg > $d/out.txt 2> $d/err.txt || { echo "run $n $leg failed"; tail -5 $d/err.txt; exit 1; }
    echo "== n $n $leg: $(cat $d/out.txt)"
    python3 tools/dropin_legs.py $d
  done
done 2>&1 | tee $O/legs.txt
