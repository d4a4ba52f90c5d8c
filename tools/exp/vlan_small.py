"""vlan_small.py — measurement tool (not product): VLAN push / pop + checksums on 1M short frames
(IPv4/UDP of length L in 128-byte slots with room for the tag), HIP events over alternating
push / pop launches (nfcs_time_vlan_device); the result digest after one push is printed so two
builds can be compared byte for byte (NFCS_LIB selects the build).
  python tools/exp/vlan_small.py [L ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

eng = nf.Engine(0)
n = 1 << 20
for L in [int(x) for x in (sys.argv[1:] or ["64", "256", "512"])]:
    slot = (L + 4 + 127) // 128 * 128
    rng = np.random.default_rng(L)
    host = rng.integers(0, 256, size=(n, slot), dtype=np.uint8)
    host[:, L:] = 0
    host[:, 12], host[:, 13], host[:, 14], host[:, 15] = 0x08, 0x00, 0x45, 0x00
    host[:, 16], host[:, 17] = (L - 14) >> 8, (L - 14) & 0xFF
    host[:, 22], host[:, 23] = 64, 17
    host[:, 38], host[:, 39] = (L - 34) >> 8, (L - 34) & 0xFF
    desc = np.zeros(n, dtype=nf.DESC_DTYPE)
    desc["off16"] = np.arange(n, dtype=np.uint32) * (slot // 16)
    desc["len"] = L
    a = eng.alloc(host.nbytes).upload(host)
    d = eng.alloc(desc.nbytes).upload(desc)
    push = nf.vlan_push_op(100, 3)
    eng.time_vlan_device(a, host.nbytes, d, n, push, nf.VLAN_POP, slot, 20)  # warm (even: back to start)
    ms = eng.time_vlan_device(a, host.nbytes, d, n, push, nf.VLAN_POP, slot, 40) / 40
    eng.vlan_device(a, host.nbytes, d, n, op_all=push, cap_all=slot)
    eng.sync()
    dig = eng.digest_device(a, host.nbytes, d, n, 0)
    print(json.dumps({"frame": L, "packets": n, "kernel_us": round(ms * 1e3, 2),
                      "Mpkt_per_s": round(n / (ms * 1e-3) / 1e6, 1), "digest_after_push": f"{dig:016x}"}),
          flush=True)
    a.free()
    d.free()
eng.close()
