# whole -m gpu suite, then the drop-in API legs at 4 and 8 ranks (storm / lat / iar / iardj)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for n in 4 8; do
  for leg in "lat 500 64" "iar 2000" "iardj 2000" "storm 20000 64"; do
    timeout -k 5 120 /opt/conda/bin/mpiexec -n $n rootless-coll-mpi-ops_amd/lib/rlo_api_bench $leg 2>/dev/null | grep mode || { echo "api $n $leg failed"; exit 1; }
  done
done
