# profile evidence for a round (tag = output dir under gpurun_out/, e.g. r5p): rocprofv3 kernel stats + FETCH_SIZE /
# WRITE_SIZE PMC (separate passes, each under its own limit) of every workload a bench `frac` is quoted for -- the
# 64 B headline storm (2^18 bcasts), the 256 B / 1 KiB / 4 KiB storms (2^16), the C3 bulk leg's 1-MiB and 64-MiB
# rounds (8 ranks, tools/bulk_probe.py) -- and kernel stats of the C4 decisions leg with LDS and HBM pending tables
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
tag=${1:-prof}
P=gpurun_out/$tag/prof
mkdir -p $P
pass() {  # name, limit, command...
  local D=$P/$1 lim=$2; shift 2
  timeout -k 10 $lim rocprofv3 --kernel-trace --stats -d $D/trace -o run -- "$@" > $D.trace.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run -- "$@" > $D.fetch.log 2>&1 && \
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $D/write -o run -- "$@" > $D.write.log 2>&1 || { echo "prof $D failed"; tail -5 $D.*.log; exit 1; }
  echo "prof $D ok"
}
for L in 64 256 1024 4096; do
  K=65536; [ $L -eq 64 ] && K=262144
  pass s$L 150 python3 tools/pmc_probe.py --len $L --k $K
done
for M in 1 64; do pass bulk$M 150 python3 tools/bulk_probe.py 0 $M 8; done
D=$P/iar_lds; timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/pmc_probe.py --iar 8 > $D.log 2>&1 || { echo "prof iar failed"; exit 1; }
D=$P/iar_ph; timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $D/trace -o run -- python3 tools/pmc_probe.py --iar 8 --pend-hbm > $D.log 2>&1 || { echo "prof iar ph failed"; exit 1; }
python3 - $P > $P/summary.txt <<'PY'
import glob, os, sys
sys.path.insert(0, "tools")
from rocpd_summary import kernel_stats, pmc
P = sys.argv[1]
for d in sorted(glob.glob(P + "/*/")):
    name = os.path.basename(d.rstrip("/"))
    for db in glob.glob(d + "trace/**/*.db", recursive=True):
        with open(P + "/" + name + "_kernel_stats.csv", "w") as f:
            f.write("name,calls,total_us,avg_us,pct\n")
            for r in kernel_stats(db):
                f.write('"%s",%d,%.3f,%.3f,%.3f\n' % r)
        for r in kernel_stats(db)[:1]:
            print("%-10s stats %s calls %d total_us %.1f avg_us %.2f" % (name, r[0][:60], r[1], r[2], r[3]))
    for c in ("fetch", "write"):
        for db in glob.glob(d + c + "/**/*.db", recursive=True):
            rows = pmc(db)
            with open(P + "/" + name + "_pmc_" + c + ".csv", "w") as f:
                f.write("dispatch,kernel,counter,value,duration_ns\n")
                for r in rows:
                    f.write('%d,"%s",%s,%.4f,%d\n' % r)
            if rows:
                last = max(r[0] for r in rows)
                v = sum(r[3] for r in rows if r[0] == last)
                print("%-10s %s last dispatch %d: %s = %.0f KiB" % (name, c, last, rows[0][2], v))
PY
cat $P/summary.txt
