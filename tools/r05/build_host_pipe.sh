#!/bin/bash
# Builds tools/r05/host_pipe (measurement tool, git-ignored; host code only). Run here.
set -euo pipefail
cd "$(dirname "$0")/../.."
hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/r05/host_pipe.hip -lpthread -o tools/r05/host_pipe
