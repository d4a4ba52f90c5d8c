"""usage.py — measurement tool (not product): condenses hipcc's -Rpass-analysis=kernel-resource-usage
remarks (stderr of a build) into one line per kernel: VGPRs, SGPRs, scratch, occupancy.
  hipcc ... -Rpass-analysis=kernel-resource-usage 2> usage.txt; python tools/r05/usage.py usage.txt"""
import re
import subprocess
import sys


def parse(text):
    out, cur = {}, None
    for line in text.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark: \s*(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split()[0]] = int(m.group(2))
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


if __name__ == "__main__":
    u = parse(open(sys.argv[1]).read())
    for k, d in zip(u, demangle(list(u))):
        v = u[k]
        d = re.sub(r"\(.*", "", d.replace("nfcs::", ""))
        print(f"{v.get('VGPRs', '?'):>4} v {v.get('TotalSGPRs', '?'):>4} s {v.get('ScratchSize', '?'):>4} scr occ {v.get('Occupancy', '?')}  {d}")
