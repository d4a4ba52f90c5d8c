#!/bin/bash
# Builds tools/r05/host_phases (measurement tool, git-ignored) against the product library. Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
/opt/rocm/lib/llvm/bin/clang++ -O2 -std=c++17 -Iinclude tools/r05/host_phases.cpp -Lnetflow_amd -l:libnfcs.so \
  -Wl,-rpath,'$ORIGIN/../../netflow_amd' -Wl,-rpath,/opt/rocm/lib -lpthread -o tools/r05/host_phases
