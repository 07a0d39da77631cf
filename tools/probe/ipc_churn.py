"""Driver of tools/probe/ipc_churn.hip: R rounds of allocate -> export -> import -> write -> close -> check -> free
between two fresh processes (no process here touches the GPU).  Prints the importer's import addresses (VA
reuse) and the exporter's stale-granule count.  usage: python tools/probe/ipc_churn.py [R] [MiB] [flavour]"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "ipc_churn")
R = sys.argv[1] if len(sys.argv) > 1 else "100"
MIB = sys.argv[2] if len(sys.argv) > 2 else "64"
FL = sys.argv[3] if len(sys.argv) > 3 else "0"

ex = subprocess.Popen([EXE, "export", R, MIB], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
im = subprocess.Popen([EXE, "import", R, FL], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
vas = []
for r in range(int(R)):
    h = ex.stdout.readline()
    if not h.startswith("HANDLE"):
        print("exporter:", h.strip())
        break
    im.stdin.write(h)
    im.stdin.flush()
    w = im.stdout.readline().split()
    if not w or w[0] != "written":
        print("importer:", w)
        break
    vas.append(w[2])
    ex.stdin.write("go\n")
    ex.stdin.flush()
im.stdin.close()
print(ex.stdout.read().strip())
ex.wait(timeout=60)
im.wait(timeout=60)
print("import VAs: %d distinct of %d rounds; first ones %s" % (len(set(vas)), len(vas), vas[:4]))
