"""patch_build.py — measurement tool (not product): builds libnfcs.so from the product sources with
literal text substitutions in the sources under netflow_amd/csrc (nfcs_kernels.hip, nfcs_api.hip,
nfcs_internal.h; each OLD must occur exactly COUNT times over them, default 1; the patched copies are
compiled together from one scratch directory, so a quoted #include finds the patched header),
so a one-line policy or shape change can be A/B-timed against the product without touching it:
  python tools/patch_build.py OUT.so 'OLD' 'NEW' ['OLD' 'NEW' ...]
  NFCS_LIB=OUT.so python bench.py --op flowkey --no-cpu
Prefix OLD with '<N>*' to require N occurrences (all replaced)."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    out, pairs = sys.argv[1], sys.argv[2:]
    if not pairs or len(pairs) % 2:
        raise SystemExit(__doc__)
    csrc = os.path.join(ROOT, "netflow_amd", "csrc")
    names = ("nfcs_kernels.hip", "nfcs_api.hip", "nfcs_internal.h")
    srcs = {f: open(os.path.join(csrc, f)).read() for f in names}
    for old, new in zip(pairs[::2], pairs[1::2]):
        cnt = 1
        if "*" in old[:4] and old.split("*", 1)[0].isdigit():
            cnt, old = int(old.split("*", 1)[0]), old.split("*", 1)[1]
        got = sum(s.count(old) for s in srcs.values())
        if got != cnt:
            raise SystemExit(f"{old!r}: {got} occurrences, expected {cnt}")
        srcs = {f: s.replace(old, new) for f, s in srcs.items()}
    with tempfile.TemporaryDirectory() as tmp:
        for f, s in srcs.items():
            open(os.path.join(tmp, f), "w").write(s)
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-mllvm", "-amdgpu-kernarg-preload-count=8",
                        "-I" + os.path.join(ROOT, "include"), "-I" + tmp,
                        os.path.join(tmp, "nfcs_kernels.hip"), os.path.join(tmp, "nfcs_api.hip"), "-o", out], check=True)


if __name__ == "__main__":
    main()
