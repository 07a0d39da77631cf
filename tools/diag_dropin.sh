mkdir -p gpurun_out
cd gpurun_out && timeout -k 5 100 /opt/conda/bin/mpiexec -n 4 ../oracle/_ref/dropin_harness t2.jsonl tests2 > t2.log 2>&1; echo "rc=$?" >> t2.log
