# drop-in decisions/s, repeated: is n=8 slower than n=12 (profiles/r2_dropin_device_judge.txt)?
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_rep.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for rep in 1 2 3; do
  for n in 4 8 12 16; do
    for m in iar iardj; do
      s=$(date +%s.%N)
      r=$(timeout -k 5 90 $M -n $n $B $m 2000 2>&1 | grep '^{') || { echo "$m n=$n rc=$?" >> $out; exit 1; }
      e=$(date +%s.%N)
      echo "rep=$rep wall=$(echo "$e - $s" | bc) $r" >> $out
    done
  done
done
cat $out
