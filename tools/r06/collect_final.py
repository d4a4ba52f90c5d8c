#!/usr/bin/env python3
"""collect_final.py — measurement bookkeeping (not product): copy one tools/r06/prof_all.sh run
(gpurun_out/<call>/) into profiles/ under a prefix: each line's bench JSON and rocprofv3 kernel stats,
the PMC log and traffic.json, and the device-resident short-burst sweep as one JSON list.
  python3 tools/r06/collect_final.py gpurun_out/r6aw r06_final2"""
import json
import os
import shutil
import sys

src, prefix = sys.argv[1], sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "profiles")
lines = ["default", "c1", "c2", "c3", "c3packed", "c4shard", "l3fwd_c1", "l3fwd_4m", "l3fwd_c3", "vlan", "flowkey"]
for name in lines:
    shutil.copy(os.path.join(src, name + ".json"), os.path.join(dst, f"{prefix}_bench_{name}.json"))
    shutil.copy(os.path.join(src, name, name + "_kernel_stats.csv"), os.path.join(dst, f"{prefix}_{name}_kernel_stats.csv"))
shutil.copy(os.path.join(src, "pmc.log"), os.path.join(dst, f"{prefix}_pmc.log"))
shutil.copy(os.path.join(src, "pmc", "traffic.json"), os.path.join(dst, f"{prefix}_traffic.json"))
burst = []
for n in (1024, 4096, 16384, 65536, 262144):
    x = json.loads(open(os.path.join(src, f"burst_dev_{n}.json")).read().strip().splitlines()[-1])
    r = x.get("roofline", {})
    burst.append({"packets": n, "us_per_call_events": round(r.get("kernel_ms", 0) * 1e3, 1),
                  "us_per_step_wall": round(x["ms_per_step"] * 1e3, 1), "frac": r.get("frac"),
                  "parity": (x.get("parity") or {}).get("match")})
json.dump(burst, open(os.path.join(dst, f"{prefix}_burst_device.json"), "w"), indent=1)
print("copied", len(lines), "lines")
