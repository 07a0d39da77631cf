# a round's evidence in one call: the -m gpu suite, the default bench line, then tools/gpu_prof.sh (kernel stats + PMC)
set -o pipefail
tag=${1:-fin}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $d/gpu_tests_$tag.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $d/gpu_tests_$tag.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $d/bench_$tag.json 2> $d/bench_$tag.err || exit $?
python3 -c "
import json; b=json.load(open('$d/bench_$tag.json'))
print('value', b['value'], 'frac', b['roofline']['frac'], 'p50', b['p50_us'], 'dec', b['decisions_per_s'], 'pool16', b['pool16_decisions_per_s'])
print('small', json.dumps(b['small_worlds']))
print('bulk', [(s['MiB'], s['round_ms'], s['hbm_frac_no_verify']) for s in b['bulk']['sizes']])
print('dropin n8', json.dumps(b['dropin_api']['n8']['ratio_vs_reference']), 'n4', json.dumps(b['dropin_api']['n4']['ratio_vs_reference']))
"
[ -n "$NO_PROF" ] || bash tools/gpu_prof.sh ${RLO_OUT:-r6}p$tag
