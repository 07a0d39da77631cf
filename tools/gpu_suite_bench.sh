# evidence: the whole -m gpu suite in one process, then the default bench (logs under gpurun_out/${RLO_OUT:-r6}/)
set -o pipefail
tag=${1:-suite}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $d/gpu_tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/gpu_tests_$tag.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > $d/bench_$tag.json 2> $d/bench_$tag.err || exit $?
cat $d/bench_$tag.json
