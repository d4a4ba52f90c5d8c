"""Debug: the deferred L3 forward on the padded fuzz batch vs the oracle; prints differing frames."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import netflow_amd as nf
import oracle
from l3_common import random_l3_case
from test_gpu_l3 import _pad_groups, run_l3

eng = nf.Engine(0)
rng = np.random.default_rng(77)
frames, table, nh = random_l3_case(41, 300_001, table_n=8)
frames = _pad_groups(frames, rng)
n = 4 * len(frames) - 1
frames = (frames * 4)[:n]
nh = np.tile(nh, 4)[:n]
arena, desc = oracle.pack_frames(frames, align=128)
ref = arena.copy()
rst = oracle.l3_forward_batch(ref, desc, nh, table)
out, st = run_l3(eng, arena, desc, nh, table)
print("status equal", np.array_equal(st, rst))
bad = []
for i in range(n):
    o, l = int(desc[i]["off16"]) * 16, int(desc[i]["len"])
    if not np.array_equal(out[o:o + ((l + 15) & ~15)], ref[o:o + ((l + 15) & ~15)]):
        bad.append(i)
        if len(bad) > 2000: break
print("bad frames", len(bad), "first", bad[:10])
for i in bad[:8]:
    o, l = int(desc[i]["off16"]) * 16, int(desc[i]["len"])
    d = np.nonzero(out[o:o + l + 16] != ref[o:o + l + 16])[0]
    g4 = i & ~3
    lens = [int(desc[j]["len"]) for j in range(g4, min(g4 + 4, n))]
    print(i, "st", hex(int(st[i])), "len", l, "group lens", lens, "nh", int(nh[i]),
          "diff at", d[:12].tolist(), "got", out[o + d[:6]].tolist(), "want", ref[o + d[:6]].tolist(),
          "orig", arena[o + d[:6]].tolist(), "sub-batch", i >> 19)
