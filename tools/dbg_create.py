import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
mode = sys.argv[1]
if mode == "torch_first":
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
from kwok_amd import engine as keng, workload
keng.load_engine_lib()
if mode == "import_only":
    import torch
    import torch.distributed
for n in (1000, 100000):
    try:
        e, fl, ph = workload.build_engine_fleet(keng.Engine, n)
        r = e.tick(workload.S0 + 30, read=False)
        print(mode, n, "ok", fl.cn, fl.cp, list(r.counters)[:4], flush=True)
        if mode == "torch_first":
            torch.cuda.synchronize()
        e.close()
    except Exception as ex:
        print(mode, n, "FAIL", ex, flush=True)
import ctypes
maps = open("/proc/self/maps").read()
print(mode, sorted(set(l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "rccl" in l)))
