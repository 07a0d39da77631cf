# hop-path iteration: latency / one-proposal decisions A/B against a baseline build, the hop profile, and
# (with "suite") the whole -m gpu suite
set -o pipefail
base=${1:-r5base}; tag=${2:-lat}
mkdir -p gpurun_out/${RLO_OUT:-r6}
out=gpurun_out/${RLO_OUT:-r6}/lat_$tag.txt
: > $out
timeout -k 10 300 python3 -u tools/lat_ab.py $base 8 256 >> $out 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/hop_prof.py 8 256 >> $out 2>&1 || exit $?
cat $out
if [ "$3" = "suite" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/${RLO_OUT:-r6}/gpu_tests_$tag.log 2>&1
  rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${RLO_OUT:-r6}/gpu_tests_$tag.log | tail -12; exit $rc
fi
