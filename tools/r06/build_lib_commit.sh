#!/bin/bash
# build_lib_commit.sh COMMIT NAME — measurement build (not product): libnfcs.so from the product sources
# as of a git commit (tools/r06/libNAME.so, for bench A/Bs through NFCS_LIB). Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
commit=$1; name=$2
d=tools/r06/pre_src/$name
mkdir -p $d/include $d/csrc
git show $commit:include/nfcs.h > $d/include/nfcs.h
for f in nfcs_kernels.hip nfcs_api.hip nfcs_internal.h; do git show $commit:netflow_amd/csrc/$f > $d/csrc/$f; done
hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mllvm -amdgpu-kernarg-preload-count=8 -I$d/include -I$d/csrc \
  $d/csrc/nfcs_kernels.hip $d/csrc/nfcs_api.hip -o tools/r06/lib$name.so
