# the default bench line (python bench.py), stderr progress kept
set -o pipefail
tag=${1:-bench}
mkdir -p gpurun_out/${RLO_OUT:-r6}
timeout -k 10 900 python3 -u bench.py > gpurun_out/${RLO_OUT:-r6}/$tag.json 2> gpurun_out/${RLO_OUT:-r6}/$tag.err || { tail -20 gpurun_out/${RLO_OUT:-r6}/$tag.err; exit 1; }
tail -3 gpurun_out/${RLO_OUT:-r6}/$tag.err
python3 - gpurun_out/${RLO_OUT:-r6}/$tag.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ["value", "ms_per_step", "p50_us", "p99_us", "decisions_per_s", "decisions_per_s_pend_hbm", "pend_hbm_cost",
        "pool16_decisions_per_s", "verified"]
print({k: d.get(k) for k in keys})
print("roofline", d["roofline"].get("frac"), d["roofline"].get("traffic"))
print("small", {k: (v.get("p50_us"), v.get("decisions_per_s")) for k, v in d.get("small_worlds", {}).items()})
print("c4", d.get("c4_vs_reference"))
print("bulk", [(s["MiB"], s["round_ms"], s.get("hbm_frac_no_verify"), s["verified"]) for s in d.get("bulk", {}).get("sizes", [])])
print("c5", {k: d.get("c5_mixed", {}).get(k) for k in ("bcast_per_s", "frac", "verified")})
print("sizes", [(s.get("payload_bytes"), s.get("bcast_per_s"), s.get("frac")) for s in d.get("payload_sizes", [])])
api = d.get("dropin_api", {})
print("api", {k: v.get("ratio_vs_reference") for k, v in api.items() if isinstance(v, dict)})
PY
