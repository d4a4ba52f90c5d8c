#!/bin/bash
# build_variant.sh NAME [hipcc defines...] — measurement build (not product): libnfcs.so from the working
# tree's csrc with extra defines (tools/r06/NAME/libnfcs.so, also tools/r06/libNAME.so for bench A/Bs) and
# a netflow_adapter_test burstbench binary linked to it (tests/cpp/_ref/netflow_adapter_test_NAME). Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
name=$1; shift
mkdir -p tools/r06/$name
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -Iinclude -Inetflow_amd/csrc "$@" \
  netflow_amd/csrc/nfcs_kernels.hip netflow_amd/csrc/nfcs_api.hip -o tools/r06/$name/libnfcs.so
cp tools/r06/$name/libnfcs.so tools/r06/lib$name.so
g++ -std=c++17 -O2 -g -rdynamic -Wall -Wno-unused-variable -Iinclude -I/root/reference/include tests/cpp/netflow_adapter_test.cpp \
  -o tests/cpp/_ref/netflow_adapter_test_$name -Ltools/r06/$name -l:libnfcs.so \
  -Wl,-rpath,"\$ORIGIN/../../../tools/r06/$name" -Wl,-rpath,/opt/rocm/lib
