# N=1 bench (all legs) + a 2-process rehearsal of the N>1 path on the one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err && \
RLO_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-extras --ranks 64 --k 16384 > gpurun_out/bench2.log 2> gpurun_out/bench2.err
