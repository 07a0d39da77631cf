# host -> kernel -> host round trips through the BAR, per host CPU placement (tools/probe/bar_pingpong.hip)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bar_probe.txt
: > $out
P=tools/probe/bar_pingpong
for cpu in -1 -1 -1 -1 -1 -1 0 128; do
  echo "== cpu $cpu" >> $out
  timeout -k 5 60 $P $cpu 5000 >> $out 2>&1 || { echo "rc=$?" >> $out; exit 1; }
done
cat $out
