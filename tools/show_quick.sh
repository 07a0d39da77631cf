#!/bin/bash
# print the results of tools/gpu_quick.sh runs: bash tools/show_quick.sh tag...
for T in "$@"; do
  tail -1 gpurun_out/${T}_tests.log
  python -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('$T', 'bcast/s', round(d['bcast_per_s']), 'frac', d['roofline']['frac'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'dec/s', round(d['decisions_per_s']))" 2>/dev/null
  tail -1 gpurun_out/${T}_ss.log 2>/dev/null
done
