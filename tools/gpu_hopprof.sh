# rocprofv3 kernel stats of the hop kernel: the latency program at 8 and 256 ranks, one-proposal decisions at 8, and
# the 8-rank legs again in one-XCD worlds (RLO_PART_ONE_XCD)
set -o pipefail
d=gpurun_out/${RLO_OUT:-r6}/hopprof
mkdir -p $d
export TMPDIR=/tmp
for leg in "lat8 tools/lat_run.py 8 2000 3" "lat256 tools/lat_run.py 256 500 3" "c4n8 tools/c4_run.py 8 256 3" \
           "lat8x tools/lat_run.py 8 2000 3 one_xcd" "c4n8x tools/c4_run.py 8 256 3 one_xcd"; do
  set -- $leg
  tag=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $d/$tag -o run -- python3 "$@" > $d/$tag.log 2>&1 || exit $?
  grep -E "^n " $d/$tag.log
  python3 tools/rocpd_summary.py stats $(find $d/$tag -name "run_results.db" | head -1) > $d/${tag}_kernel_stats.csv || exit $?
  cat $d/${tag}_kernel_stats.csv
done
