# round-4 evidence, call 2: rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE PMC (separate passes, each under
# its own limit) of every workload a bench `frac` is quoted for: the 64 B headline storm (2^18 bcasts), the
# 256 B / 1 KiB / 4 KiB storms (2^16), and the C3 bulk leg's 64-MiB rounds (8 ranks, tools/bulk_probe.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r4/prof
for L in 64 256 1024 4096; do
  K=65536; [ $L -eq 64 ] && K=262144
  D=gpurun_out/r4/prof/s$L
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/pmc_probe.py --len $L --k $K > $D.trace.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- python3 tools/pmc_probe.py --len $L --k $K > $D.fetch.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- python3 tools/pmc_probe.py --len $L --k $K > $D.write.log 2>&1 || { echo "prof $L failed"; tail -5 $D.*.log; exit 1; }
  echo "prof $L ok"
done
D=gpurun_out/r4/prof/bulk64
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/bulk_probe.py 0 64 8 > $D.trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- python3 tools/bulk_probe.py 0 64 8 > $D.fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- python3 tools/bulk_probe.py 0 64 8 > $D.write.log 2>&1 || { echo "prof bulk failed"; tail -5 $D.*.log; exit 1; }
echo "prof bulk ok"
