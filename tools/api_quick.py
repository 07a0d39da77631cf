"""Quick drop-in probe: bench.py's drop-in API leg (tools/api_bench.c over librootless_ops.so beside the
compiled reference under host MPI) at 4 and 8 ranks, one JSON line per world size."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = bench.dropin_api_leg()
for k in ("n4", "n8"):
    rec = out.get(k, {})
    print(k, json.dumps({"ratio": rec.get("ratio_vs_reference"),
                         "ours": {m: {x: v for x, v in (rec.get("ours", {}).get(m) or {}).items() if x in ("p50_us", "decisions_per_s", "bcast_per_s", "error")} for m in ("lat", "iar", "iardj", "iarpool", "storm")},
                         "ref": {m: {x: v for x, v in (rec.get("reference_host_mpi", {}).get(m) or {}).items() if x in ("p50_us", "decisions_per_s", "bcast_per_s", "error")} for m in ("lat", "iar", "storm")}}), flush=True)
