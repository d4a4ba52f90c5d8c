"""Measurement builds (not product): the fused forward's short-mix shape as 16-lane rows in one-wave
workgroups at 7 waves/SIMD (the plain update's short shape), with buffer loads (fwd16buf) or global
loads (fwd16), segment stores past the caches — against the product's 8-lane rows of 12 slots.
Copies the product sources to a temporary directory, applies the edits, builds
tools/r05/lib<variant>.so through build_lib.sh. Run here: python3 tools/r05/fwd16_exp.py."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
SRC = os.path.join(ROOT, "netflow_amd", "csrc")

EDITS = {
    "launch": ("launch_rows<12, 8, 6, 64, true, SF_INLINE, 1, 12>((n + 7u) / 8u,",
               "launch_rows<6, 16, 7, 64, true, SF_INLINE, 0, 6>((n + 3u) / 4u,"),
    "nt": ("if (R == 8 && LA) st16_nt((uint4*)frame + rl, v);",
           "if ((R == 8 && LA) || (R == 16 && !LA)) st16_nt((uint4*)frame + rl, v);"),
    "buf": ("constexpr bool BUF = !FWD && BS == 64 && R == 16;",
            "constexpr bool BUF = BS == 64 && R == 16;"),
}
VARIANTS = {"fwd16buf": ["launch", "nt", "buf"], "fwd16": ["launch", "nt"]}

for name, edits in VARIANTS.items():
    tmp = tempfile.mkdtemp()
    for f in ("nfcs_kernels.hip", "nfcs_api.hip", "nfcs_internal.h"):
        shutil.copy(os.path.join(SRC, f), tmp)
    p = os.path.join(tmp, "nfcs_kernels.hip")
    s = open(p).read()
    for e in edits:
        a, b = EDITS[e]
        assert s.count(a) == 1, (name, e)
        s = s.replace(a, b)
    open(p, "w").write(s)
    subprocess.run(["bash", os.path.join(ROOT, "tools/r05/build_lib.sh"), f"tools/r05/lib{name}.so"],
                   env=dict(os.environ, SRC=tmp), check=True, cwd=ROOT)
    shutil.rmtree(tmp)
    print(name, open(os.path.join(ROOT, f"tools/r05/lib{name}.usage.txt")).read()[:2000])
