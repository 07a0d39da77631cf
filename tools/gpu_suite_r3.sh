set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r3_gpu_tests.log
exit $rc
