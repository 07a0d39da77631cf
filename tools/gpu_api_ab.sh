# drop-in A/B: the product build against tools/ab_libs/* on one box, legs interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 tools/api_ab.py --reps 3 2>&1 | tee gpurun_out/r3_api_ab.txt
