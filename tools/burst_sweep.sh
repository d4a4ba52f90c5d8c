#!/bin/bash
# Per-call rate of nfcs_update_device by burst size (C1 frames, device-resident): bench.py --packets P.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/burst
for p in 1024 4096 16384 65536 262144 1048576; do
  timeout -k 10 120 python3 bench.py --packets $p --steps 50 --warmup 10 --no-cpu --no-fresh > gpurun_out/burst/p$p.json 2> gpurun_out/burst/p$p.err || exit 1
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/burst/p$p.json')); print($p, d['ms_per_step'], d['value'], d['roofline']['kernel_ms'], d['parity']['match'])"
done
