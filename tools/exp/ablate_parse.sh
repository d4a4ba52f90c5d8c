#!/bin/bash
# Measurement build (not product): the launch forms of tools/exp/nfcs_exp.hip with the header parse
# removed — row_process's fast_plan call replaced by a fixed IPv4/UDP plan computed from the length
# alone (stores at bytes 24-25 and 40-41, region [34, len)) — as tools/exp/libnfcs_abl.so. Output
# digests are wrong by construction; only the timing means anything. Run here, then on the box:
#   NFCS_LIB=tools/exp/libnfcs_abl.so python tools/exp/ab.py --variants 0,2,5 --work c3,c1
# (profiles/r02_s3_c3_parse_ablation.jsonl).
set -e
cd "$(dirname "$0")/../.."
tmp=$(mktemp -d)
python3 - "$tmp" <<'EOF'
import sys
tmp = sys.argv[1]
call = "RPlan P = fast_plan<R>(h0, rowbase4, len);"
s = open("netflow_amd/csrc/nfcs_kernels.hip").read()
assert call in s, "row_process no longer calls fast_plan this way"
s = s.replace(call, "RPlan P = rplan_none(NFCS_ST_V4_UDP); P.flags = F_IP | F_L4 | F_UDP; "
              "P.ipw = 24u | (0x1234u << 16); P.rs = 34u; P.re = len > 42u ? len : 0u; P.fs = 40u; "
              "P.corr = h0.x & 0xFFu;")
open(f"{tmp}/nfcs_kernels.hip", "w").write(s)
e = open("tools/exp/nfcs_exp.hip").read()
e = e.replace('#include "../../netflow_amd/csrc/nfcs_kernels.hip"', f'#include "{tmp}/nfcs_kernels.hip"')
open(f"{tmp}/nfcs_exp.hip", "w").write(e)
EOF
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Iinclude -Inetflow_amd/csrc \
  "$tmp/nfcs_exp.hip" netflow_amd/csrc/nfcs_api.hip -o tools/exp/libnfcs_abl.so
rm -rf "$tmp"
