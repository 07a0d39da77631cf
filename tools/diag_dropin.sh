mkdir -p gpurun_out
cd gpurun_out && timeout -k 5 100 /opt/conda/bin/mpiexec -n 4 ../oracle/_ref/dropin_harness t1.jsonl tests > t1.log 2>&1; echo "rc=$?" >> t1.log
