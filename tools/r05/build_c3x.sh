#!/bin/bash
# build_c3x.sh — measurement build (not product): the product kernels + tools/r05/c3_exp.hip's C3 write
# schedules + the product C ABI, as tools/r05/libnfcs_c3x.so (git-ignored). Run here, not on the box.
set -euo pipefail
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude \
  -Inetflow_amd/csrc tools/r05/c3_exp.hip netflow_amd/csrc/nfcs_api.hip -o tools/r05/libnfcs_c3x.so \
  -Rpass-analysis=kernel-resource-usage 2> tools/r05/libnfcs_c3x.remarks
python3 tools/r05/usage.py tools/r05/libnfcs_c3x.remarks | grep -E "c3_fused|apply_records|6, 16, 7, 64"
rm -f tools/r05/libnfcs_c3x.remarks
