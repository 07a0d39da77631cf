# rocprofv3 evidence for the payload-size legs (C2 at 256 B and 4 KiB, 65,536 bcasts over 256 ranks):
# kernel trace + stats, then one PMC pass per counter (FETCH_SIZE, WRITE_SIZE), each under its own limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_sizes
for L in 256 4096; do
  D=gpurun_out/prof_sizes/s$L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/pmc_probe.py --len $L --k 65536 > $D.trace.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- python3 tools/pmc_probe.py --len $L --k 65536 > $D.fetch.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- python3 tools/pmc_probe.py --len $L --k 65536 > $D.write.log 2>&1 || { echo "prof $L failed"; tail -5 $D.*.log; exit 1; }
  echo "prof $L ok"
done
