# drop-in n=8 iardj: which leg of a proposal holds the ~1 ms stalls (RLO_TRACE leg histograms)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_legs.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for rep in 1 2 3 4 5 6 7 8 9 10; do
  echo "== rep $rep" >> $out
  RLO_HOST_DIAG=1 RLO_TRACE=1 RLO_PROXY_DIAG=1 timeout -k 5 90 $M -n 8 $B iardj 2000 >> $out 2>&1 || { echo "rc=$?" >> $out; exit 1; }
done
grep -E "^==|split|hdiag rank 0|mode" $out
