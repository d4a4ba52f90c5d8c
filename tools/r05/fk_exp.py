"""Measurement builds (not product): the flow-key kernel's header-line loads with other cache
policies — `nt` (fk_nt), `sc1` (fk_sc1), `sc0 sc1` (fk_sc), `sc0 sc1 nt` (fk_scnt) — against the
default policy, to see whether the L2 then fetches less than a whole 128-byte line per frame (the
kernel needs bytes 0..47 of most frames) and whether that raises the packet rate. Builds
tools/r05/lib<variant>.so through build_lib.sh. Run here: python3 tools/r05/fk_exp.py."""
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
SRC = os.path.join(ROOT, "netflow_amd", "csrc")
LOAD = "        c[k] = ld16<0>((rl < 3u && rl * 16u < ql) ? src + rl : zl);\n"
AFTER = "#pragma unroll\n    for (uint32_t k = 0; k < 8; ++k)\n        if (rl < 3u) *(uint4*)(rows + (8u * k + r) * kFkRow + 16u * rl) = c[k];\n"


def asm_load(pol):
    return ("        {\n"
            "            const uint4* a_ = (rl < 3u && rl * 16u < ql) ? src + rl : zl;\n"
            "            u32x4_t t_;\n"
            f"            asm volatile(\"global_load_dwordx4 %0, %1, off {pol}\" : \"=v\"(t_) : \"v\"(a_) : \"memory\");\n"
            "            c[k] = make_uint4(t_.x, t_.y, t_.z, t_.w);\n"
            "        }\n")


VARIANTS = {
    "fk_nt": (LOAD.replace("ld16<0>", "ld16<1>"), False),
    "fk_sc1": (asm_load("sc1"), True),
    "fk_sc": (asm_load("sc0 sc1"), True),
    "fk_scnt": (asm_load("sc0 sc1 nt"), True),
}

for name, (load, wait) in VARIANTS.items():
    tmp = tempfile.mkdtemp()
    for f in ("nfcs_kernels.hip", "nfcs_api.hip", "nfcs_internal.h"):
        shutil.copy(os.path.join(SRC, f), tmp)
    p = os.path.join(tmp, "nfcs_kernels.hip")
    s = open(p).read()
    assert s.count(LOAD) == 1 and s.count(AFTER) == 1
    s = s.replace(LOAD, load)
    if wait:
        s = s.replace(AFTER, "    asm volatile(\"s_waitcnt vmcnt(0)\" ::: \"memory\");\n" + AFTER)
    open(p, "w").write(s)
    subprocess.run(["bash", os.path.join(ROOT, "tools/r05/build_lib.sh"), f"tools/r05/lib{name}.so"],
                   env=dict(os.environ, SRC=tmp), check=True, cwd=ROOT)
    shutil.rmtree(tmp)
    for line in open(os.path.join(ROOT, f"tools/r05/lib{name}.usage.txt")):
        if "flow_keys" in line:
            print(name, line.strip())
