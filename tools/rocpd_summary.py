"""Summarise rocprofv3 rocpd databases (ROCm 7.2 writes SQLite by default).

  python tools/rocpd_summary.py stats <run_results.db>          -> kernel stats CSV (name, calls, total_us, avg_us, pct)
  python tools/rocpd_summary.py pmc <run_results.db> [kernel]   -> per-dispatch counters CSV

Used by bench.py (live PMC traffic) and to produce the summaries committed under profiles/.
"""
import sqlite3
import sys


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    c.close()
    return rows


def pmc(db, kernel_like="%rlo_progress%"):
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection "
                     "where kernel_name like ? order by dispatch_id", (kernel_like,)).fetchall()
    c.close()
    return rows


def main():
    what, db = sys.argv[1], sys.argv[2]
    if what == "stats":
        print("name,calls,total_us,avg_us,pct")
        for r in kernel_stats(db):
            print('"%s",%d,%.3f,%.3f,%.3f' % r)
    else:
        print("dispatch,kernel,counter,value,duration_ns")
        for r in pmc(db, sys.argv[3] if len(sys.argv) > 3 else "%rlo_progress%"):
            print('%d,"%s",%s,%.4f,%d' % r)


if __name__ == "__main__":
    main()
