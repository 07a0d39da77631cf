# GPU check of the working tree: the whole -m gpu suite, then a bench run without the slow legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests rc=$?"; grep -E "FAIL|Error|error" gpurun_out/gpu_tests.log | head -20; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 400 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-api --no-bulk --no-pmc > gpurun_out/bench_quick.json 2> gpurun_out/bench_quick.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_quick.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_quick.json'))
print('value', d['value'], 'frac', d['roofline']['frac'], 'dec', d.get('decisions_per_s'), 'pool16', d.get('pool16_decisions_per_s'))
print(json.dumps(d.get('small_worlds')))"
bash tools/gpu_api_pool.sh
