#!/bin/bash
# Inline vs deferred stores by uniform frame length (tools/exp/ab.py work u<L>), replayed and fresh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/lensweep
for f in 1 3; do
  timeout -k 10 300 python tools/exp/ab.py --variants 1,4,2,3 --work u256,u512,u768,u1024,u1280,u1500 \
    --lds 24576 --fresh $f >> gpurun_out/lensweep/ab.jsonl 2>&1 || exit 1
done
cat gpurun_out/lensweep/ab.jsonl
