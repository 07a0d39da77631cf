set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu_pull_ab.sh
