# Diagnostic A/B beyond 8 rank processes: previous drop-in (tools/old_lib) vs shared host service,
# with an 8-rank control for box noise and an idle queue-holding torch process beside 8 ranks.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/ab2.txt
: > $out
M=/opt/conda/bin/mpiexec
NEW=rootless-coll-mpi-ops_amd/lib/rlo_api_bench
OLD=tools/old_lib/rlo_api_bench
run() {  # label exe n
  timeout -k 5 ${T:-70} $M -n $3 $2 iar 2000 > gpurun_out/o.json 2>/dev/null
  echo "$1 n=$3 rc=$? $(tail -1 gpurun_out/o.json)" >> $out
}
run OLD $OLD 8; run NEW $NEW 8
run NEW $NEW 9; run NEW $NEW 12; run NEW $NEW 16
run OLD $OLD 9
run OLD $OLD 8; run NEW $NEW 8
rm -f gpurun_out/dummy_ready
timeout -k 5 100 python3 -c "
import torch, time
x = torch.ones(1, device='cuda'); torch.cuda.synchronize()
open('gpurun_out/dummy_ready', 'w').close(); time.sleep(80)" &
dummy=$!
for i in $(seq 90); do [ -f gpurun_out/dummy_ready ] && break; sleep 1; done
run OLD_beside_torch $OLD 8; run NEW_beside_torch $NEW 8; run NEW_beside_torch $NEW 12
kill $dummy 2>/dev/null; wait $dummy 2>/dev/null
exit 0
