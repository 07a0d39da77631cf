"""bench.py's drop-in API leg alone (tools/api_bench.c over librootless_ops.so beside the compiled reference),
with the KFD census and CPU-quota throttling per run:  python3 tools/api_leg.py [ranks ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ranks = tuple(int(x) for x in sys.argv[1:]) or (4, 8)
print(json.dumps(bench.dropin_api_leg(ranks=ranks)), flush=True)
