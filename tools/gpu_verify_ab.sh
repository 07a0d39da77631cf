# A/B of the bulk VERIFY job's cost: the product build, the checksum without the per-granule generator comparison
# (lib_vnocmp), and the read-back alone (lib_vread: fails verification by design) -- 8 ranks, 1 / 4 / 64 MiB
set -o pipefail
d=gpurun_out/${RLO_OUT:-r6}
mkdir -p $d
out=$d/verify_ab.txt
: > $out
for rep in 1 2; do
  for lib in lib lib_vnocmp lib_vread; do
    echo "== $lib rep $rep" >> $out
    if [ $lib = lib ]; then timeout -k 10 200 python3 -u tools/bulk_probe.py 0 1,4,64 8 >> $out 2>&1 || exit $?
    else RLO_LIB_DIR=$lib timeout -k 10 200 python3 -u tools/bulk_probe.py 0 1,4,64 8 >> $out 2>&1 || echo "($lib: exit $?)" >> $out; fi
  done
done
cat $out
