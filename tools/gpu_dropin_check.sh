# GPU check of the drop-in (shared host service): its parity tests, iar at 8 / 12 / 16 ranks on one
# GPU (one queue-holding process per GPU whatever the rank count), and a KFD census during a run.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_check.txt
: > $out
df -h /dev/shm >> $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
timeout -k 5 60 $M -n 4 $B iar 2000 >> $out 2>&1 || { echo "iar n=4 failed rc=$?" >> $out; exit 1; }
timeout -k 10 ${TESTS_T:-600} python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_dropin.py > gpurun_out/dropin_tests.log 2>&1
echo "dropin tests rc=$?" >> $out
for n in 8 12 16; do
  timeout -k 5 90 $M -n $n $B iar 2000 >> $out 2>&1 || { echo "iar n=$n failed rc=$?" >> $out; exit 1; }
done
timeout -k 5 90 $M -n 12 $B iar 40000 > gpurun_out/o12.json 2>&1 &
bg=$!
sleep 3
for d in /sys/class/kfd/kfd/proc/*; do
  p=$(basename $d); echo "kfd pid $p queues $(ls $d/queues 2>/dev/null | wc -l) cmd $(tr '\0' ' ' < /proc/$p/cmdline 2>/dev/null | cut -c1-60)" >> $out
done
echo "rank processes: $(pgrep -c rlo_api_bench)" >> $out
wait $bg; echo "iar40000 n=12 rc=$? $(tail -1 gpurun_out/o12.json)" >> $out
for n in 8 12; do
  timeout -k 5 90 $M -n $n $B storm 20000 64 >> $out 2>&1 || { echo "storm n=$n failed" >> $out; exit 1; }
  timeout -k 5 90 $M -n $n $B lat 500 64 >> $out 2>&1 || { echo "lat n=$n failed" >> $out; exit 1; }
done
