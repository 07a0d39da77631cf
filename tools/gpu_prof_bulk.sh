# rocprofv3 kernel stats of the C3 bulk leg's workload (8 ranks on one GPU, 64 MiB rounds of the latency program)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_bulk
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bulk/trace -o run -- python3 tools/bulk_probe.py 0 64 8 > gpurun_out/prof_bulk/trace.log 2>&1
rc=$?; tail -3 gpurun_out/prof_bulk/trace.log; exit $rc
