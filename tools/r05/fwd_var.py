"""fwd_var.py — measurement tool (not product): where the fused forward's run-to-run spread on BASELINE
C3's mix comes from. One process: --allocs times, generate 2 separately allocated 4M-frame C3 batches
(fresh device memory each time), then --windows timing windows of --iters forwards rotating over them
(HIP events on the engine's stream, TTLs restored before each window), then free them. If windows within
one allocation agree and allocations differ, the spread follows where the frames sit in memory.
One JSON line per window.  NFCS_LIB=... python3 tools/r05/fwd_var.py --allocs 4 --windows 3
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402  (torch's HIP runtime first, as bench.py does)

torch.cuda.set_device(0)
torch.cuda.init()
import netflow_amd as nf  # noqa: E402

SEED = 20250620


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--allocs", type=int, default=4)
    ap.add_argument("--windows", type=int, default=3)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--op", default="l3fwd", choices=["l3fwd", "update"])
    a = ap.parse_args()
    eng = nf.Engine(0)
    n = 1 << 22
    g3 = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))["l3fwd_c1"]
    table = np.frombuffer(bytes.fromhex(g3["table"]), dtype=np.uint8).copy()
    d_tab = eng.alloc(table.nbytes).upload(table)
    d_nh = eng.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
    st = torch.cuda.ExternalStream(eng.stream)
    for al in range(a.allocs):
        bs = [eng.config_batch(3, SEED, 0, n, 128)[:3] for _ in range(2)]
        frame_bytes = None
        for w in range(a.windows):
            for ar, nb, de in bs:
                eng.gen_config_device(3, SEED, 0, n, ar, nb, de)
            eng.sync()
            for k in range(6):  # warm
                ar, nb, de = bs[k % 2]
                (eng.l3_forward_device(ar, nb, de, d_nh, n, d_tab, 8) if a.op == "l3fwd" else eng.update_device(ar, nb, de, n))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for k in range(a.iters):
                ar, nb, de = bs[k % 2]
                (eng.l3_forward_device(ar, nb, de, d_nh, n, d_tab, 8) if a.op == "l3fwd" else eng.update_device(ar, nb, de, n))
            e1.record(st)
            e1.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            print(json.dumps({"op": a.op, "alloc": al, "window": w, "ms_per_call": round(ms, 4),
                              "arena_ptrs": [hex(b[0].ptr) for b in bs]}), flush=True)
        for ar, _, de in bs:
            ar.free()
            de.free()


if __name__ == "__main__":
    main()
