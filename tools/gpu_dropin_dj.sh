# drop-in: parity tests (incl. the device-judge multi-proposal cases) and iar vs iardj at 4/8/12 ranks
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dropin_dj.txt
: > $out
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
M=/opt/conda/bin/mpiexec
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_dropin.py > gpurun_out/dropin_tests.log 2>&1
echo "dropin tests rc=$? $(tail -1 gpurun_out/dropin_tests.log)" >> $out
for n in 4 8 12; do
  for m in iar iardj; do
    timeout -k 5 90 $M -n $n $B $m 2000 >> $out 2>&1 || { echo "$m n=$n rc=$?" >> $out; exit 1; }
  done
done
for n in 4 8; do timeout -k 5 90 $M -n $n oracle/_ref/ref_api_bench iar 2000 >> $out 2>&1 || exit 1; done
