#!/bin/bash
# Round-4 measurement build: the product kernels + tools/r04/fresh_exp.hip's launch forms + the product
# C ABI, as tools/r04/libnfcs_r4.so (git-ignored). Run here (CPU container), not on the box.
set -e
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -Inetflow_amd/csrc \
  tools/r04/fresh_exp.hip netflow_amd/csrc/nfcs_api.hip -o tools/r04/libnfcs_r4.so
