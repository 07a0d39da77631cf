# the storm's per-phase cycles at every rank (tools/diag.py, MODE_PROF in the diagnostics build), 64 B and 256 B
set -o pipefail
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
RLO_DIAG_LIB=1 timeout -k 10 300 python3 -u tools/diag.py --n 256 --lens 64,256 --storm-only > $d/storm_diag_${1:-a}.txt 2>&1 || exit $?
cat $d/storm_diag_${1:-a}.txt
timeout -k 10 300 python3 -u tools/api_ab.py --reps 3 --ranks 4 8 -- rootless-coll-mpi-ops_amd/lib > $d/api_ab_${1:-a}.txt 2>&1 || exit $?
cat $d/api_ab_${1:-a}.txt
