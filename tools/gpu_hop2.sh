# hop-kernel quick iteration: the section anatomy (diagnostics build) and the latency / decisions A/B
set -o pipefail
base=${1:-r6h1}; tag=${2:-hq}
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
timeout -k 10 120 python3 -u tools/hop_anatomy.py 8 > $d/anat_$tag.txt 2>&1 || exit $?
cat $d/anat_$tag.txt
timeout -k 10 300 python3 -u tools/lat_ab.py $base 4 8 > $d/lat_$tag.txt 2>&1 || exit $?
cat $d/lat_$tag.txt
