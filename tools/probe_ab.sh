# Diagnostic A/B: the previous drop-in (tools/old_lib: one persistent kernel per rank process) vs the
# shared host service (one leader process per GPU), alternating in one box session; thread / CPU
# placement snapshots during one run of each.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab.txt
: > $out
M=/opt/conda/bin/mpiexec
NEW=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
OLD=tools/old_lib/rlo_api_bench
snap() {  # label
  sleep 1.5
  echo "--- snapshot $1" >> $out
  ps -eLo pid,tid,psr,pcpu,stat,comm --sort=-pcpu | head -40 >> $out
  for p in $(pgrep rlo_api_bench); do echo "pid $p $(grep Cpus_allowed_list /proc/$p/status)" >> $out; done
}
for i in 1 2 3 4; do
  for v in OLD NEW; do
    exe=${!v}
    timeout -k 5 40 $M -n 8 $exe iar 2000 > gpurun_out/o.json 2>/dev/null
    echo "$v run $i rc=$? $(tail -1 gpurun_out/o.json)" >> $out
  done
done
for v in OLD NEW; do
  exe=${!v}
  timeout -k 5 40 $M -n 8 $exe iar 20000 > gpurun_out/o.json 2>/dev/null &
  bg=$!
  snap $v
  wait $bg
  echo "$v long rc=$? $(tail -1 gpurun_out/o.json)" >> $out
done
exit 0
