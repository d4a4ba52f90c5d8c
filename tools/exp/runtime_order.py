"""Measurement tool (not product): which HIP runtime torch and libnfcs.so end up on, by load order.
  python tools/exp/runtime_order.py engine-first | torch-first"""
import sys

order = sys.argv[1] if len(sys.argv) > 1 else "engine-first"
sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
if order == "torch-first":
    import torch
    torch.cuda.init()
import netflow_amd as nf  # noqa: E402
e = nf.Engine(0)
import torch  # noqa: E402
print(order, "is_available", torch.cuda.is_available())
try:
    torch.cuda.synchronize()
    print(order, "torch.cuda.synchronize OK")
except Exception as ex:  # noqa: BLE001
    print(order, "torch.cuda.synchronize FAILED:", str(ex)[:80])
maps = open("/proc/self/maps").read()
print(order, "runtimes mapped:", sorted({l.split()[-1] for l in maps.splitlines() if "libamdhip64" in l}))
e.close()
