"""slot_hint.py — measurement tool (not product): a burst of 1M short frames (IPv4/UDP of length L
in 128-byte-aligned slots) at the start of a 4 GiB arena, as in a NIC ring: the checksum update and VLAN
push/pop timed by HIP events (nfcs_time_*_device) with the arena deciding the launch shape
(arena_bytes / n = 4 KiB: 16-lane rows), with the slot-size hint (nfcs_ctx_set_slot_bytes = the slot:
8-lane rows), and over an exact-size arena; digests printed so the three can be compared.
  python tools/exp/slot_hint.py [L ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import netflow_amd as nf  # noqa: E402

eng = nf.Engine(0)
n = 1 << 20
RING = 4 << 30
for L in [int(x) for x in (sys.argv[1:] or ["64", "256"])]:
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
    a = eng.alloc(RING)
    d = eng.alloc(desc.nbytes).upload(desc)
    for name, arena_bytes, hint in (("ring", RING, 0), ("ring+hint", RING, slot), ("exact", host.nbytes, 0)):
        eng.set_slot_bytes(hint)
        a.upload(host)
        eng.time_update_device(a, arena_bytes, d, n, 20)
        us = eng.time_update_device(a, arena_bytes, d, n, 40) / 40 * 1e3
        dig = eng.digest_device(a, host.nbytes, d, n, 0)
        a.upload(host)
        push = nf.vlan_push_op(100, 3)
        eng.time_vlan_device(a, arena_bytes, d, n, push, nf.VLAN_POP, slot, 20)
        vus = eng.time_vlan_device(a, arena_bytes, d, n, push, nf.VLAN_POP, slot, 40) / 40 * 1e3
        print(json.dumps({"frame": L, "packets": n, "arena": name, "slot_hint": hint,
                          "update_us": round(us, 2), "update_digest": f"{dig:016x}",
                          "vlan_us": round(vus, 2)}), flush=True)
    eng.set_slot_bytes(0)
    a.free()
    d.free()
eng.close()
