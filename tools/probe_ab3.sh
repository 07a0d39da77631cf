# Diagnostic: the shared host service after registering the segment MTYPE_UC -- repeats of the cases
# that were erratic (n=8 beside an idle torch process, n=12), with the previous design as control.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab3.txt
: > $out
M=/opt/conda/bin/mpiexec
NEW=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
OLD=tools/old_lib/rlo_api_bench
run() {  # label exe n
  timeout -k 5 ${T:-60} $M -n $3 $2 iar 2000 > gpurun_out/o.json 2>/dev/null
  echo "$1 n=$3 rc=$? $(tail -1 gpurun_out/o.json)" >> $out
}
run OLD $OLD 8
for i in 1 2 3; do run NEW $NEW 8; run NEW $NEW 12; run NEW $NEW 16; done
rm -f gpurun_out/dummy_ready
timeout -k 5 150 python3 -c "
import torch, time
x = torch.ones(1, device='cuda'); torch.cuda.synchronize()
open('gpurun_out/dummy_ready', 'w').close(); time.sleep(130)" &
dummy=$!
for i in $(seq 90); do [ -f gpurun_out/dummy_ready ] && break; sleep 1; done
for i in 1 2 3; do run NEW_beside_torch $NEW 8; run NEW_beside_torch $NEW 12; done
kill $dummy 2>/dev/null; wait $dummy 2>/dev/null
run OLD $OLD 8
exit 0
