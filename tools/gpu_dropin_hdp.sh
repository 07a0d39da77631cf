# HDP flush A/B for the drop-in (BAR stores the kernel polls): n=8 iardj / iar, alternating
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_hdp.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for rep in 1 2 3 4 5; do
  for ab in flush noflush; do
    for m in iardj iar; do
      if [ $ab = noflush ]; then export RLO_NO_HDP_FLUSH=1; else unset RLO_NO_HDP_FLUSH; fi
      r=$(API_DIAG=1 timeout -k 5 90 $M -n 8 $B $m 2000 2> gpurun_out/hdp_diag_$ab.txt | grep '^{') || { echo "$ab $m rc=$?" >> $out; exit 1; }
      p99=$(grep -o "p99 [0-9.]*" gpurun_out/hdp_diag_$ab.txt | awk '{if ($2>m) m=$2} END {print m}')
      echo "$ab rep=$rep max_rank_p99_us=$p99 $r" >> $out
    done
  done
done
unset RLO_NO_HDP_FLUSH
for n in 4 12 16; do
  for m in iardj iar; do
    r=$(timeout -k 5 90 $M -n $n $B $m 2000 2>/dev/null | grep '^{') || { echo "n=$n $m rc=$?" >> $out; exit 1; }
    echo "flush n=$n $r" >> $out
  done
done
cat $out
