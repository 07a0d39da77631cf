# the whole -m gpu suite (one process), then the box's CPU share for the record
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r3_gpu_tests.log | tail -25
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/r3_box_cpus.txt 2>&1
exit $rc
