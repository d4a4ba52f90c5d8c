"""exp_build.py — measurement tool (not product): builds a measurement library from a tools/r04
experiment translation unit (default fresh_exp.hip, which #includes the product kernels) and the product
C ABI, with literal text substitutions applied to copies of the product sources first (as
tools/patch_build.py does for the product library). Used for ablations: timing-only builds whose
bytes are wrong on purpose, never loaded by tests or bench.py.
  python tools/r04/exp_build.py OUT.so [--exp tools/r04/fresh_exp.hip] ['OLD' 'NEW' ...]
  NFCS_LIB=OUT.so python3 tools/r04/fresh_forms.py --variants 14,15 --work c3
Prefix OLD with '<N>*' to require N occurrences (all replaced)."""
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REV = "00f5686"  # the round-4 final tree
ROOT = os.path.dirname(os.path.dirname(HERE))


def main():
    args = sys.argv[1:]
    if not args:
        raise SystemExit(__doc__)
    out, args = args[0], args[1:]
    exp = os.path.join(HERE, "fresh_exp.hip")
    if args[:1] == ["--exp"]:
        exp, args = os.path.abspath(args[1]), args[2:]
    if len(args) % 2:
        raise SystemExit(__doc__)
    names = ("nfcs_kernels.hip", "nfcs_api.hip", "nfcs_internal.h")
    # fresh_exp.hip instantiates round 4's row_stage / row_process (its COLD and KC knobs, dropped from
    # the product in round 5): the product sources as of the round-4 final tree, from git
    srcs = {f: subprocess.run(["git", "-C", ROOT, "show", f"{REV}:netflow_amd/csrc/{f}"], check=True,
                              capture_output=True, text=True).stdout for f in names}
    for old, new in zip(args[::2], args[1::2]):
        cnt = 1
        if "*" in old[:4] and old.split("*", 1)[0].isdigit():
            cnt, old = int(old.split("*", 1)[0]), old.split("*", 1)[1]
        got = sum(s.count(old) for s in srcs.values())
        if got != cnt:
            raise SystemExit(f"{old!r}: {got} occurrences, expected {cnt}")
        srcs = {f: s.replace(old, new) for f, s in srcs.items()}
    with tempfile.TemporaryDirectory() as tmp:
        # the experiment file includes "../../netflow_amd/csrc/nfcs_kernels.hip": mirror that layout
        d_csrc = os.path.join(tmp, "netflow_amd", "csrc")
        d_exp = os.path.join(tmp, "tools", "r04")
        os.makedirs(d_csrc)
        os.makedirs(d_exp)
        for f, s in srcs.items():
            open(os.path.join(d_csrc, f), "w").write(s)
        e = os.path.join(d_exp, os.path.basename(exp))
        open(e, "w").write(open(exp).read())
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-mllvm",
                        "-amdgpu-kernarg-preload-count=8", "-I" + os.path.join(ROOT, "include"), "-I" + d_csrc,
                        e, os.path.join(d_csrc, "nfcs_api.hip"), "-o", out], check=True)


if __name__ == "__main__":
    main()
