import os, sys, json
sys.path.insert(0, os.getcwd())
from mpi_blockchain_amd.miner import GpuMiner
n = int(sys.argv[1]); th = sys.argv[2] == "1"
ms = [GpuMiner(0, test_hooks=th) for _ in range(n)]
for m in ms: m.warmup()
b = ms[0]
from mpi_blockchain_amd.block import make_block
for m in ms: m.mine(make_block(1,0,9,1700000000,b""), 0, 1<<16, 9)
d = f"/sys/class/kfd/kfd/proc/{os.getpid()}/queues"
q = sorted(os.listdir(d)) if os.path.isdir(d) else None
info = {}
if q:
    for x in q:
        p = os.path.join(d, x)
        info[x] = {f: open(os.path.join(p, f)).read().strip() for f in os.listdir(p) if os.path.isfile(os.path.join(p, f))}
print(json.dumps({"contexts": n, "test_lib": th, "env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES","POW_AQL")}, "kfd_queues": len(q) if q is not None else "no sysfs", "detail": info}))
