mkdir -p gpurun_out; : > gpurun_out/hiar.log
B=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
echo "# pump" >> gpurun_out/hiar.log; RLO_TRACE=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n 8 $B iar 300 >> gpurun_out/hiar.log 2>&1
echo "# nopump" >> gpurun_out/hiar.log; RLO_NO_PUMP=1 RLO_TRACE=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n 8 $B iar 300 >> gpurun_out/hiar.log 2>&1
echo "# nopump 6" >> gpurun_out/hiar.log; RLO_NO_PUMP=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n 6 $B iar 300 >> gpurun_out/hiar.log 2>&1
echo "# nopump 8 bind" >> gpurun_out/hiar.log; RLO_NO_PUMP=1 timeout -k 5 60 /opt/conda/bin/mpiexec -bind-to core -n 8 $B iar 300 >> gpurun_out/hiar.log 2>&1
nproc >> gpurun_out/hiar.log; cat /sys/fs/cgroup/cpu.max >> gpurun_out/hiar.log 2>&1; taskset -p $$ >> gpurun_out/hiar.log 2>&1
