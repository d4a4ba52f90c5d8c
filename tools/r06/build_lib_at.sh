#!/bin/bash
# build_lib_at.sh NAME REV [hipcc defines...] — measurement build (not product): libnfcs.so from the csrc of
# git revision REV (tools/r06/NAME/libnfcs.so) and a netflow_amd_test burstbench binary linked to it
# (tests/cpp/_ref/netflow_adapter_test_NAME), for A/B runs of the host path. Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
name=$1 rev=$2; shift 2
src=tools/r06/$name/src
mkdir -p "$src"
for f in nfcs_api.hip nfcs_kernels.hip nfcs_internal.h; do git show "$rev:netflow_amd/csrc/$f" > "$src/$f"; done
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -I"$src" "$@" \
  "$src/nfcs_kernels.hip" "$src/nfcs_api.hip" -o tools/r06/$name/libnfcs.so
g++ -std=c++17 -O2 -g -rdynamic -Wall -Wno-unused-variable -Iinclude -I/root/reference/include tests/cpp/netflow_adapter_test.cpp \
  -o tests/cpp/_ref/netflow_adapter_test_$name -Ltools/r06/$name -l:libnfcs.so \
  -Wl,-rpath,"\$ORIGIN/../../../tools/r06/$name" -Wl,-rpath,/opt/rocm/lib
