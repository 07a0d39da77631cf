# the 8-part rehearsal of bench.py --gpus 8 on one GPU (tests/test_gpu_multigpu.py::test_bench_eight_parts_under_torchrun's
# command), its stderr kept: python's progress lines and, with RLO_DEBUG_REGIONS=1, every part's exported regions
set -o pipefail
tag=${1:-r8}
mkdir -p gpurun_out/${RLO_OUT:-r6}
RLO_BENCH_DEVICE=0 MASTER_ADDR=127.0.0.1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 8 --steps 2 --warmup 1 --ranks 32 --k 16384 --lat-rounds 200 \
  --no-api --no-pmc --no-cpu-baseline > gpurun_out/${RLO_OUT:-r6}/$tag.out 2> gpurun_out/${RLO_OUT:-r6}/$tag.err
rc=$?
grep -E "exports|as mapped here|leg failed" gpurun_out/${RLO_OUT:-r6}/$tag.err | cut -c1-260 | head -120
tail -c 600 gpurun_out/${RLO_OUT:-r6}/$tag.out
exit $rc
