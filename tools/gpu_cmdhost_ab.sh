# command path in host memory (default) vs through the BAR (RLO_BAR_CMDS=1): parity, then n=8 A/B
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/cmdhost_ab.txt
: > $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > gpurun_out/cmdhost_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/cmdhost_tests.log; exit 1; }
tail -1 gpurun_out/cmdhost_tests.log >> $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
for rep in 1 2 3; do
  for ab in host bar; do
    if [ $ab = bar ]; then export RLO_BAR_CMDS=1; else unset RLO_BAR_CMDS; fi
    for leg in "iardj 2000" "iar 2000" "lat 500 64"; do
      r=$(timeout -k 5 90 $M -n 8 $B $leg 2>/dev/null | grep '^{') || { echo "$ab $leg rc=$?" >> $out; exit 1; }
      echo "$ab rep=$rep $r" >> $out
    done
  done
done
unset RLO_BAR_CMDS
for n in 4 12 16; do
  r=$(timeout -k 5 90 $M -n $n $B iardj 2000 2>/dev/null | grep '^{') || { echo "n=$n rc=$?" >> $out; exit 1; }
  echo "host n=$n $r" >> $out
done
cat $out
