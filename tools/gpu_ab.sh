# A/B of this tree's library against a baseline build (tools/ab_libs/<base>, lib_<base>/):
# latency + one-proposal decisions (tools/lat_ab.py), the 256-rank storms (tools/storm_ab.py) and the 8-rank
# bulk rounds (tools/bulk_probe.py), interleaved
set -o pipefail
base=${1:-r5base}; tag=${2:-ab}
mkdir -p gpurun_out/${RLO_OUT:-r6}
out=gpurun_out/${RLO_OUT:-r6}/ab_$tag.txt
: > $out
timeout -k 10 300 python3 -u tools/lat_ab.py $base 8 256 >> $out 2>&1 || exit $?
for rep in 1 2; do
  timeout -k 10 200 python3 -u tools/storm_ab.py >> $out 2>&1 || exit $?
  RLO_LIB_DIR=lib_$base timeout -k 10 200 python3 -u tools/storm_ab.py >> $out 2>&1 || exit $?
  echo "bulk head" >> $out; timeout -k 10 200 python3 -u tools/bulk_probe.py 0 1,4,64 8 >> $out 2>&1 || exit $?
  echo "bulk $base" >> $out; RLO_LIB_DIR=lib_$base timeout -k 10 200 python3 -u tools/bulk_probe.py 0 1,4,64 8 >> $out 2>&1 || exit $?
done
cat $out
