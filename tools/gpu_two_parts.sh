# The two-part torchrun bench on one GPU, timed, with its stderr kept (tests/test_gpu_multigpu.py).
set -o pipefail
mkdir -p gpurun_out
export RLO_BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1
start=$(date +%s)
timeout -k 10 ${T:-200} python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --ranks 64 --k 16384 --lat-rounds 200 --no-api \
  --no-pmc --no-cpu-baseline > gpurun_out/two_parts.json 2> gpurun_out/two_parts.err
rc=$?
echo "rc=$rc elapsed=$(( $(date +%s) - start ))s"
tail -c 3000 gpurun_out/two_parts.err
exit $rc
