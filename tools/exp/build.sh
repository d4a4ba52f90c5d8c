#!/bin/bash
# Measurement build: the product kernels + the extra launch forms of tools/exp/nfcs_exp.hip + the
# product C ABI, as tools/exp/libnfcs_exp.so (git-ignored). Run here (CPU container), not on the box.
set -e
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -Inetflow_amd/csrc \
  tools/exp/nfcs_exp.hip netflow_amd/csrc/nfcs_api.hip -o tools/exp/libnfcs_exp.so
