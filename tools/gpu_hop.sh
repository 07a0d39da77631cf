# hop-kernel iteration: the latency / iar tests, A/B of latency + one-proposal decisions against a baseline build
# (tools/ab_libs/<base>), the latency-round timeline of the hop kernel (diagnostics build)
set -o pipefail
base=${1:-r6h1}; tag=${2:-hop}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_timeline.py -m gpu -x -v --timeout 120 --timeout-method thread > $d/tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/tests_$tag.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/lat_ab.py $base 4 8 256 > $d/lat_$tag.txt 2>&1 || exit $?
cat $d/lat_$tag.txt
timeout -k 10 120 python3 -u tools/round_timeline.py --n 8 --sizes 64 --rounds 64 > $d/tl_$tag.txt 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/hop_anatomy.py 8 256 > $d/anat_$tag.txt 2>&1 || exit $?
cat $d/anat_$tag.txt
tail -4 $d/tl_$tag.txt
