# one hop-path iteration on the box: the -m gpu suite, the hop/full A/B, the latency-round timelines of both kernels
# and a short default bench (everything under gpurun_out/${RLO_OUT:-r6}/, tagged $1)
set -o pipefail
tag=${1:-it}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $d/gpu_tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/gpu_tests_$tag.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/hop_ab.py 4 8 64 256 > $d/hop_ab_$tag.txt 2>&1 || exit $?
cat $d/hop_ab_$tag.txt
timeout -k 10 120 python3 -u tools/round_timeline.py --n 8 --sizes 64 --rounds 64 > $d/tl_hop_$tag.txt 2>&1 || exit $?
RLO_NO_HOP=1 timeout -k 10 120 python3 -u tools/round_timeline.py --n 8 --sizes 64 --rounds 64 > $d/tl_full_$tag.txt 2>&1 || exit $?
tail -25 $d/tl_hop_$tag.txt; tail -25 $d/tl_full_$tag.txt
timeout -k 10 300 python3 -u bench.py > $d/bench_$tag.json 2> $d/bench_$tag.err || exit $?
cat $d/bench_$tag.json
