# writer-wave A/B (drop-in legs, product lib vs lib_nowq), the latency-round timelines with global-pointer probes, the
# -m gpu suite and a bench run (under gpurun_out/${RLO_OUT:-r6}/, tagged $1)
set -o pipefail
tag=${1:-it2}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
[ -n "$SKIP_SUITE" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $d/gpu_tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/gpu_tests_$tag.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u tools/api_ab.py --reps 3 --ranks 4 8 -- rootless-coll-mpi-ops_amd/lib rootless-coll-mpi-ops_amd/lib_nowq > $d/api_ab_$tag.txt 2>&1 || exit $?
cat $d/api_ab_$tag.txt
timeout -k 10 120 python3 -u tools/round_timeline.py --n 8 --sizes 64 --rounds 64 > $d/tl_hop_$tag.txt 2>&1 || exit $?
RLO_NO_HOP=1 timeout -k 10 120 python3 -u tools/round_timeline.py --n 8 --sizes 64 --rounds 64 > $d/tl_full_$tag.txt 2>&1 || exit $?
tail -3 $d/tl_hop_$tag.txt; tail -3 $d/tl_full_$tag.txt
timeout -k 10 300 python3 -u bench.py > $d/bench_$tag.json 2> $d/bench_$tag.err || exit $?
python3 -c "
import json,sys; b=json.load(open('$d/bench_$tag.json'))
print('value', b['value'], 'p50', b['p50_us'], 'dec', b['decisions_per_s'], 'pool16', b['pool16_decisions_per_s'])
print('small', json.dumps(b['small_worlds']))
print('dropin n8', json.dumps(b['dropin_api']['n8']['ratio_vs_reference']), 'n4', json.dumps(b['dropin_api']['n4']['ratio_vs_reference']))
"
