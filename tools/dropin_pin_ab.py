"""DESIGN 4.2's open hypothesis, tested: does where the drop-in's rank processes run (relative to the GPU's NUMA
node) explain the 8-rank spread and the host-judge decision rate?  Runs tools/api_bench.c over librootless_ops.so
(the bench's API leg, ours only) with the rank processes unpinned, pinned one per core on the GPU's NUMA node,
and pinned on another node, interleaved, `reps` times each.   python3 tools/dropin_pin_ab.py [ranks] [reps]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "rootless-coll-mpi-ops_amd", "lib", "rlo_api_bench")
MPIEXEC = "/opt/conda/bin/mpiexec"
nr = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3


def cpulist(s):
    out = []
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


# the GPU this box gives us (a child process: this one never touches the GPU)
q = subprocess.run([sys.executable, "-c", "import torch; p = torch.cuda.get_device_properties(0); "
                    "print('%04x:%02x:%02x.0' % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id))"],
                   capture_output=True, text=True, timeout=300)
bus = q.stdout.strip().splitlines()[-1] if q.stdout.strip() else ""
node = -1
try:
    node = int(open("/sys/bus/pci/devices/%s/numa_node" % bus).read())
except Exception:  # noqa: BLE001
    pass
avail = sorted(os.sched_getaffinity(0))
nodes = {}
for d in sorted(os.listdir("/sys/devices/system/node")):
    if d.startswith("node") and d[4:].isdigit():
        nodes[int(d[4:])] = [c for c in cpulist(open("/sys/devices/system/node/%s/cpulist" % d).read()) if c in avail]
print(json.dumps({"gpu_bus": bus, "gpu_numa_node": node, "nodes": {k: len(v) for k, v in nodes.items()}}), flush=True)
near = nodes.get(node, [])[:nr]
far_node = next((k for k in nodes if k != node and len(nodes[k]) >= nr), None)
far = nodes[far_node][:nr] if far_node is not None else []
configs = [("unpinned", [])]
if len(near) == nr:
    configs.append(("near", ["-bind-to", "user:" + ",".join(map(str, near))]))
if len(far) == nr:
    configs.append(("far", ["-bind-to", "user:" + ",".join(map(str, far))]))
# whole NUMA nodes (every thread of every rank process may run on any CPU of the node: the app thread, its pump
# thread and the leader's proxy thread), by the affinity mpiexec and its children inherit
if nodes.get(node):
    configs.append(("near-node", ["@taskset", ",".join(map(str, nodes[node]))]))
if far_node is not None:
    configs.append(("far-node", ["@taskset", ",".join(map(str, nodes[far_node]))]))
legs = [("storm", ["storm", "20000", "64"]), ("iar", ["iar", "2000"]), ("lat", ["lat", "500", "64"])]
res = {}
for rep in range(reps):
    for name, bind in configs:
        for leg, args in legs:
            if bind and bind[0] == "@taskset":
                cmd = ["timeout", "-k", "5", "150", "taskset", "-c", bind[1], MPIEXEC, "-n", str(nr), EXE] + args
            else:
                cmd = ["timeout", "-k", "5", "150", MPIEXEC] + bind + ["-n", str(nr), EXE] + args
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
            lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
            d = json.loads(lines[-1]) if lines else {"error": "rc=%d %s" % (r.returncode, r.stderr[-200:])}
            key = {"storm": "bcast_per_s", "iar": "decisions_per_s", "lat": "p50_us"}[leg]
            res.setdefault(name, {}).setdefault(leg, []).append(d.get(key, d.get("error")))
            print("rep %d %-9s %-5s %s" % (rep, name, leg, d.get(key, d.get("error"))), flush=True)
print(json.dumps({"ranks": nr, "gpu_numa_node": node, "near_cpus": near, "far_cpus": far, "results": res}), flush=True)
