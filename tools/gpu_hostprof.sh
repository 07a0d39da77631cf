# the host service's doorbell passes (diagnostics build, RLO_HOP_PROF): one bcast at a time in one process
# (tools/hop_prof.py --host), then the drop-in's lat / iar / iardj legs at 8 ranks, whose leader prints the part's
# pass profile and why passes handed over to the full iteration
set -o pipefail
O=gpurun_out/${RLO_OUT:-r6}/hostprof; mkdir -p $O
timeout -k 10 200 python3 -u tools/hop_prof.py 8 --host 2>&1 | tee $O/hop_host.txt || exit 1
B=rootless-coll-mpi-ops_amd/lib_diag/rlo_api_bench
for leg in "lat 500 64" "iar 2000" "iardj 2000"; do
  RLO_NUMA_BIND=all RLO_HOP_PROF=1 timeout -k 5 120 /opt/conda/bin/mpiexec -n 8 $B $leg > $O/out.txt 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
  echo "== $leg: $(cat $O/out.txt)"; grep "hopprof" $O/err.txt
done 2>&1 | tee -a $O/hop_host.txt
