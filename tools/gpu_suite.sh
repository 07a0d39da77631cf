# evidence: the whole -m gpu suite in one process (log under gpurun_out/${RLO_OUT:-r6}/)
set -o pipefail
mkdir -p gpurun_out/${RLO_OUT:-r6}
tag=${1:-suite}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${RLO_OUT:-r6}/gpu_tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${RLO_OUT:-r6}/gpu_tests_$tag.log | tail -12; exit $rc
