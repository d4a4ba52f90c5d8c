#!/bin/bash
# Measurement build (not product): the launch forms of tools/exp/nfcs_exp.hip with the read pass's
# inline checksum byte stores (row_process's emit) issued with one cache policy in every shape, as
# tools/exp/libnfcs_stp.so. The bytes written are the product's; only the policy bits differ. (The
# product: `sc0 sc1 nt` in the short-frame shape, `sc1` elsewhere; profiles/r02_s3_inline_store_policy_ab.jsonl.)
#   tools/exp/store_policy.sh "sc1"
#   NFCS_LIB=tools/exp/libnfcs_stp.so python tools/exp/ab.py --variants 0 --work c3,imix
set -e
cd "$(dirname "$0")/../.."
pol="${1:-sc1}"
tmp=$(mktemp -d)
python3 - "$tmp" "$pol" <<'PYEOF'
import sys
tmp, pol = sys.argv[1], sys.argv[2]
old = """if (NT) st8_nt(frame + pos, w >> (16 + 8 * (rl & 1u)));
                else st8<true>(frame + pos, w >> (16 + 8 * (rl & 1u)));"""
s = open("netflow_amd/csrc/nfcs_kernels.hip").read()
assert s.count(old) == 1, "row_process's inline store changed"
s = s.replace(old, "asm volatile(\"global_store_byte %0, %1, off " + pol
              + "\" :: \"v\"(frame + pos), \"v\"(w >> (16 + 8 * (rl & 1u))) : \"memory\");")
open(f"{tmp}/nfcs_kernels.hip", "w").write(s)
e = open("tools/exp/nfcs_exp.hip").read()
e = e.replace('#include "../../netflow_amd/csrc/nfcs_kernels.hip"', f'#include "{tmp}/nfcs_kernels.hip"')
open(f"{tmp}/nfcs_exp.hip", "w").write(e)
PYEOF
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Iinclude -Inetflow_amd/csrc \
  "$tmp/nfcs_exp.hip" netflow_amd/csrc/nfcs_api.hip -o tools/exp/libnfcs_stp.so
rm -rf "$tmp"
