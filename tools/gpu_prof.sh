# rocprofv3 evidence for the bench workload: kernel trace + stats, then one PMC pass per counter group
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline --no-api --no-bulk --no-pmc > gpurun_out/prof/bench_trace.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run -- python3 tools/pmc_probe.py > gpurun_out/prof/fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run -- python3 tools/pmc_probe.py > gpurun_out/prof/write.log 2>&1
