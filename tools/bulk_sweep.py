"""Sweep the bulk bcast's chunk count and workgroups per rank on one GPU (8-rank world).

    python tools/bulk_sweep.py > gpurun_out/bulk_sweep.jsonl

Prints one JSON line per (MiB, chunks, blocks): median kernel ms over 5 launches (rotating
originators, first launch a warmup) and whether every receiver got every byte.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rootless-coll-mpi-ops_amd"))

import torch  # noqa: E402

import rlo  # noqa: E402
from rlo.bulk import Bulk  # noqa: E402

G = int(os.environ.get("RLO_SWEEP_RANKS", "8"))


def main():
    sizes = [1, 4, 16, 64]
    w = rlo.World(G, max_payload=64, device=0)
    b = Bulk(w, max(sizes) << 20)
    b.connect([b.export()])
    try:
        for mib in sizes:
            nbytes = mib << 20
            want = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device="cuda")
            for blocks in (0, 32, 64, 128):
                for k in ((0,) if blocks == 0 else (1, 2, 4, 8, 16)):
                    ms_l, ok = [], True
                    for it in range(6):
                        o = it % G
                        b.tensor(o)[:nbytes].copy_(want)
                        torch.cuda.synchronize()
                        b.reset()
                        b.launch(o, nbytes, blocks=blocks, chunk=(nbytes + k - 1) // k if k else 0)
                        ms, rc = b.wait(raise_on_error=False)
                        ok &= rc == 0
                        for r in range(G):
                            if r != o:
                                ok &= bool(torch.equal(b.tensor(r)[:nbytes], want))
                        if it:
                            ms_l.append(ms)
                    ms = sorted(ms_l)[len(ms_l) // 2]
                    print(json.dumps({"MiB": mib, "chunks": k or "default", "blocks": blocks or "auto", "ms": round(ms, 4),
                                      "algbw_GBps": round(nbytes / ms / 1e6, 1), "ok": ok}), flush=True)
                    if not ok:
                        return 1
    finally:
        b.close()
        w.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
