# SQ counters of the hop kernel on the C4 workload (8 ranks): instructions by kind and wait cycles, one pass
set -o pipefail
d=gpurun_out/${RLO_OUT:-r6}/c4pmc
mkdir -p $d
export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/c4_run.py 8 256 3 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d $d/a -o run -- python3 tools/c4_run.py 8 256 1 > $d/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $d/b -o run -- python3 tools/c4_run.py 8 256 1 > $d/b.log 2>&1 || exit $?
find $d -name "*.csv" | head
