#!/bin/bash
# build_fwdb.sh — measurement build (not product): the product kernels + tools/r06/fwd_bound.hip's
# forward-bound probes + the product C ABI, as tools/r06/libnfcs_fwdb.so (git-ignored). Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude \
  -Inetflow_amd/csrc tools/r06/fwd_bound.hip netflow_amd/csrc/nfcs_api.hip -o tools/r06/libnfcs_fwdb.so \
  -Rpass-analysis=kernel-resource-usage 2> tools/r06/libnfcs_fwdb.remarks
python3 tools/r05/usage.py tools/r06/libnfcs_fwdb.remarks | grep -E "fwd_rw|12, 8, 6, 256" || true
rm -f tools/r06/libnfcs_fwdb.remarks
