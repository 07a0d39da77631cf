set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/apid.jsonl; : > $out; : > gpurun_out/apid.err
for cfg in "8 storm 500 64" "6 storm 2000 64" "8 storm 2000 64"; do
  set -- $cfg; n=$1; shift
  echo "# ours n=$n $*" >> $out
  timeout -k 5 40 /opt/conda/bin/mpiexec -n $n rootless-coll-mpi-ops_amd/lib/rlo_api_bench $* >> $out 2>> gpurun_out/apid.err
  echo "rc=$?" >> $out
done
