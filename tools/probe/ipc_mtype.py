"""Driver of tools/probe/ipc_mtype.hip (VERDICT r4 "next" 1): the memory type of a hipIpc-imported mapping,
seen through what a writer in ANOTHER process leaves stale at the owner.  Every process is started fresh
(no process here touches the GPU); usage: python tools/probe/ipc_mtype.py [K]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "ipc_mtype")
K = sys.argv[1] if len(sys.argv) > 1 else "200"


def cross(alloc, flavour):
    ex = subprocess.Popen([EXE, "export", alloc, K], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    line = ex.stdout.readline().split()
    assert line and line[0] == "HANDLE", line
    im = subprocess.run([EXE, "import", line[1], str(flavour), K], capture_output=True, text=True, timeout=120)
    out, _ = ex.communicate("done\n", timeout=120)
    print(im.stdout.strip() or im.stderr.strip())
    print(out.strip())


def local(alloc, flavour):
    r = subprocess.run([EXE, "local", alloc, str(flavour), K], capture_output=True, text=True, timeout=120)
    print((r.stdout + r.stderr).strip())


for alloc in ("uncached", "cached"):
    for f in range(4):
        print("== %s allocation, flavour %d" % (alloc, f), flush=True)
        local(alloc, f)
        cross(alloc, f)
