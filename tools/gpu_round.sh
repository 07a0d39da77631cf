# round-end evidence, one call: the whole -m gpu suite (one process), the default bench line, then
# rocprofv3 kernel stats of the bench workload and one PMC pass per counter (FETCH_SIZE, WRITE_SIZE)
set -o pipefail
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_gpu_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
tail -2 gpurun_out/r3_bench.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-extras --no-cpu-baseline --no-api --no-bulk --no-pmc > gpurun_out/prof/bench_trace.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/fetch -o run -- python3 tools/pmc_probe.py > gpurun_out/prof/fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/write -o run -- python3 tools/pmc_probe.py > gpurun_out/prof/write.log 2>&1
