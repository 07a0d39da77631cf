set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_dj.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for n in 4 8 12; do
  for m in iar iardj; do
    timeout -k 5 90 $M -n $n $B $m 2000 >> $out 2>&1 || { echo "$m n=$n rc=$?" >> $out; exit 1; }
  done
done
for n in 4 8; do timeout -k 5 90 $M -n $n oracle/_ref/ref_api_bench iar 2000 >> $out 2>&1 || exit 1; done
