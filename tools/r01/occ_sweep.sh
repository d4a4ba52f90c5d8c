#!/bin/bash
# Occupancy sweep through dynamic LDS padding (NFCS_LDS_PAD bytes per 256-thread workgroup;
# 160 KiB LDS per CU => 4 waves of one workgroup per CU-quarter: pad P allows floor(160K/P)
# workgroups per CU = that many waves per SIMD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "$@"; do  # variant:pad:benchargs
  IFS=: read -r v pad args <<< "$spec"
  NFCS_VARIANT=$v NFCS_LDS_PAD=$pad timeout -k 10 120 python bench.py $args --steps 30 --warmup 3 --no-cpu > /tmp/o.json 2>/dev/null || { echo "fail $spec"; exit 1; }
  python3 -c "import json; d=json.loads(open('/tmp/o.json').read()); print('$spec', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'], d['parity']['match'])"
done
