#!/bin/bash
# Round-4 measurement build: the product kernels + tools/r04/fresh_exp.hip's launch forms + the product
# C ABI, as tools/r04/libnfcs_r4.so (git-ignored). Run here (CPU container), not on the box.
# fresh_exp.hip instantiates round 4's row_stage / row_process, so the product sources come from the
# round-4 final tree (git 00f5686), as tools/r04/exp_build.py takes them.
set -e
cd "$(dirname "$0")/../.."
exec python3 tools/r04/exp_build.py tools/r04/libnfcs_r4.so
