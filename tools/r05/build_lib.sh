#!/bin/bash
# build_lib.sh OUT.so [hipcc args...] — measurement build (not product): the product sources as they are
# in netflow_amd/csrc (or SRC=dir), with extra hipcc arguments (e.g. -DNFCS_DATA_PAD=4096), and a
# resource-usage summary beside the library (OUT.usage.txt). Run here, in the CPU container.
set -euo pipefail
cd "$(dirname "$0")/../.."
out=$1; shift
src=${SRC:-netflow_amd/csrc}
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -I"$src" \
  "$@" "$src/nfcs_kernels.hip" "$src/nfcs_api.hip" -o "$out" -Rpass-analysis=kernel-resource-usage 2> "$out.remarks"
python3 tools/r05/usage.py "$out.remarks" > "${out%.so}.usage.txt"
rm -f "$out.remarks"
