#!/bin/bash
# Measurement build (not product): libnfcs.so with its 16-byte write-through stores (st16<true>: the
# fused L3 forward's header segment and the VLAN kernel's frame rewrite) issued with another cache
# policy, as tools/exp/libnfcs_st16.so; the bytes written are the product's. Compare with
#   NFCS_LIB=tools/exp/libnfcs_st16.so python bench.py --op l3fwd|vlan --no-cpu
#   tools/exp/wide_store_policy.sh "sc0 sc1 nt"      (the product: sc1)
set -e
cd "$(dirname "$0")/../.."
pol="${1:-sc0 sc1 nt}"
tmp=$(mktemp -d)
python3 - "$tmp" "$pol" <<'PYEOF'
import sys
tmp, pol = sys.argv[1], sys.argv[2]
old = 'asm volatile("global_store_dwordx4 %0, %1, off sc1\\n\\ts_nop 1" ::"v"(p), "v"(t) : "memory");'
s = open("netflow_amd/csrc/nfcs_kernels.hip").read()
assert s.count(old) == 1, "st16's store changed"
s = s.replace(old, old.replace("off sc1", "off " + pol))
open(f"{tmp}/nfcs_kernels.hip", "w").write(s)
PYEOF
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Iinclude -Inetflow_amd/csrc \
  "$tmp/nfcs_kernels.hip" netflow_amd/csrc/nfcs_api.hip -o tools/exp/libnfcs_st16.so
rm -rf "$tmp"
