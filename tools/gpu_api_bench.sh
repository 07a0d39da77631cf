# drop-in API bench (ours on the GPU, the reference on the host cores), one JSON line per run
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/api.jsonl; : > $out
for n in ${RANKS:-4 8}; do
  for m in "storm 20000 64" "lat 500 64" "iar 2000"; do
    echo "# ours n=$n $m" >> $out
    timeout -k 5 120 /opt/conda/bin/mpiexec -n $n rootless-coll-mpi-ops_amd/lib/rlo_api_bench $m >> $out 2>> gpurun_out/api.err || exit 1
    echo "# reference n=$n $m" >> $out
    timeout -k 5 120 /opt/conda/bin/mpiexec -n $n oracle/_ref/ref_api_bench $m >> $out 2>> gpurun_out/api.err || exit 1
  done
done
