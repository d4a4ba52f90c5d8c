"""Debug (not a test): frames where the write-through VLAN kernel differs from the oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import netflow_amd as nf
import oracle
from vlan_common import vlan_fixture

z, frames = vlan_fixture()
arena, desc = oracle.pack_frames(frames, align=16, room=4)
ref = arena.copy()
rst = oracle.vlan_batch(ref, desc.copy(), z["ops"], z["caps"])
with nf.Engine(0) as e:
    n = len(desc)
    da = e.alloc(arena.nbytes).upload(arena); dd = e.alloc(desc.nbytes).upload(desc)
    do = e.alloc(4 * n).upload(np.ascontiguousarray(z["ops"], np.uint32))
    dc = e.alloc(4 * n).upload(np.ascontiguousarray(z["caps"], np.uint32))
    ds = e.alloc(n)
    e.vlan_device(da, arena.nbytes, dd, n, do, 0, dc, 0, ds); e.sync()
    out = da.download(np.uint8, arena.nbytes); st = ds.download(np.uint8, n)
diff = np.nonzero(out != ref)[0]
print("bytes differing:", len(diff), "status equal:", np.array_equal(st, rst))
offs = desc["off16"].astype(np.int64) * 16
idx = np.searchsorted(offs, diff, side="right") - 1
seen = {}
for b, i in zip(diff, idx):
    seen.setdefault(int(i), []).append(int(b - offs[i]))
for i in list(seen)[:12]:
    f = frames[i]
    print(f"frame {i}: len {len(f)} op {int(z['ops'][i]):#x} cap {int(z['caps'][i])} st {int(st[i]):#x} ref_st {int(rst[i]):#x} "
          f"tagged {f[12:14] == bytes([0x81, 0])} ihl {f[14] & 15 if len(f) > 14 else -1} diff at {seen[i][:8]} "
          f"got {[int(out[offs[i] + o]) for o in seen[i][:4]]} want {[int(ref[offs[i] + o]) for o in seen[i][:4]]} in {[int(arena[offs[i] + o]) for o in seen[i][:4]]}")
