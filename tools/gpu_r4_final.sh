# round-4 end evidence: the whole -m gpu suite (one process), the default bench line, and rocprofv3 kernel stats +
# FETCH_SIZE / WRITE_SIZE PMC (separate passes, each under its own limit) of the 64 B headline storm and the C3 bulk
# leg's 1-MiB and 64-MiB rounds at HEAD
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4f/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r4f/gpu_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r4f/gpu_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 560 python3 -u bench.py > gpurun_out/r4f/bench.json 2> gpurun_out/r4f/bench.err || { tail -20 gpurun_out/r4f/bench.err; exit 1; }
tail -2 gpurun_out/r4f/bench.err
D=gpurun_out/r4f/prof/s64
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/pmc_probe.py --len 64 --k 262144 > $D.trace.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- python3 tools/pmc_probe.py --len 64 --k 262144 > $D.fetch.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- python3 tools/pmc_probe.py --len 64 --k 262144 > $D.write.log 2>&1 || { echo "prof 64 failed"; exit 1; }
for M in 1 64; do
  D=gpurun_out/r4f/prof/bulk$M
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/bulk_probe.py 0 $M 8 > $D.trace.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- python3 tools/bulk_probe.py 0 $M 8 > $D.fetch.log 2>&1 && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- python3 tools/bulk_probe.py 0 $M 8 > $D.write.log 2>&1 || { echo "prof bulk $M failed"; exit 1; }
done
echo "prof ok"
