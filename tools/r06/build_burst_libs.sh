#!/bin/bash
# build_burst_libs.sh — measurement builds (not product) for the per-RX-burst A/B of round 6 (calls.sh f):
# libnfcs.so from the sources before direct chunks (tools/r06/pre_src, git a4256f8), and the product
# sources with NFCS_DIRECT_CHUNK_BYTES = 0 (no direct chunk) and 8 MiB, each with its own
# netflow_adapter_test burstbench binary linked to it (tests/cpp/_ref/netflow_adapter_test_<name>).
set -euo pipefail
cd "$(dirname "$0")/../.."
# the sources before direct chunks, from git (not kept in the tree)
mkdir -p tools/r06/pre_src
for f in nfcs_api.hip nfcs_kernels.hip nfcs_internal.h; do git show a4256f8:netflow_amd/csrc/$f > tools/r06/pre_src/$f; done
HIPCC="hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude"
one() {  # one NAME SRC [defines]
  local name=$1 src=$2; shift 2
  mkdir -p tools/r06/$name
  $HIPCC -I"$src" "$@" "$src/nfcs_kernels.hip" "$src/nfcs_api.hip" -o tools/r06/$name/libnfcs.so
  g++ -std=c++17 -O2 -g -rdynamic -Wall -Wno-unused-variable -Iinclude -I/root/reference/include tests/cpp/netflow_adapter_test.cpp \
    -o tests/cpp/_ref/netflow_adapter_test_$name -Ltools/r06/$name -l:libnfcs.so \
    -Wl,-rpath,"\$ORIGIN/../../../tools/r06/$name" -Wl,-rpath,/opt/rocm/lib
}
one pre tools/r06/pre_src &
one d0 netflow_amd/csrc -DNFCS_DIRECT_CHUNK_BYTES=0 &
one d8 netflow_amd/csrc -DNFCS_DIRECT_CHUNK_BYTES="(8u<<20)" &
wait
