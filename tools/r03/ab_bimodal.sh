#!/bin/bash
# Round 3: the product (short shape defers groups of 4 averaging >= 1280 B to a write pass) against
# inline-only short/tiny shapes (c3inl) on 4M-frame mixes of 64- and 1500-byte frames (tools/r03/bimodal.py).
set -o pipefail
out=gpurun_out/${1:-r03_ab_bimodal}
mkdir -p $out
for f in 0.5 0.75 0.25; do
for r in 1 2; do
for lib in tools/exp/libnfcs_prev.so tools/exp/libnfcs_c3inl.so; do
  NFCS_LIB=$lib timeout -k 10 300 python3 tools/r03/bimodal.py --long-frac $f | tee -a $out/ab.jsonl || exit 1
done
done
done
