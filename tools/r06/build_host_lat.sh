#!/bin/bash
# build_host_lat.sh — measurement tool (not product): tools/r06/host_lat against the product library.
set -euo pipefail
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O2 -std=c++17 -Iinclude tools/r06/host_lat.hip -o tools/r06/host_lat \
  -Lnetflow_amd -l:libnfcs.so -Wl,-rpath,'$ORIGIN/../../netflow_amd'
