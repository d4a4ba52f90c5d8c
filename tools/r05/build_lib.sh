#!/bin/bash
# build_lib.sh OUT.so [hipcc args...] — measurement build (not product): the product sources as they are
# in netflow_amd/csrc (or SRC=dir), with extra hipcc arguments (e.g. -DNFCS_PAST=1), and a resource-usage
# summary beside the library (OUT.usage.txt). PAD=<bytes> first inserts a used __device__ array of that
# size before the kernels' globals, so the data section (and every global's address) moves. Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
out=$1; shift
src=${SRC:-netflow_amd/csrc}
if [ -n "${PAD:-}" ]; then
  tmp=$(mktemp -d); cp "$src"/nfcs_kernels.hip "$src"/nfcs_api.hip "$src"/nfcs_internal.h "$tmp"/
  python3 - "$tmp/nfcs_kernels.hip" "$PAD" <<'PY'
import sys
p, pad = sys.argv[1], int(sys.argv[2])
s = open(p).read()
anchor = "__device__ __attribute__((aligned(4096))) uint4 g_zero_line[8];"
assert s.count(anchor) == 1
s = s.replace(anchor, f"__device__ __attribute__((used)) uint8_t g_data_pad[{pad}];\n" + anchor)
open(p, "w").write(s)
PY
  src=$tmp
fi
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -I"$src" \
  "$@" "$src/nfcs_kernels.hip" "$src/nfcs_api.hip" -o "$out" -Rpass-analysis=kernel-resource-usage 2> "$out.remarks"
python3 tools/r05/usage.py "$out.remarks" > "${out%.so}.usage.txt"
rm -f "$out.remarks"
