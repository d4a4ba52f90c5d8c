#!/bin/bash
# C4 shard (4M x 1500 B on one GPU, the per-GPU work of the N > 1 line): bench line with parity,
# rocprofv3 kernel stats, PMC traffic and write requests (tools/pmc_traffic.py --packets).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 bench.py --packets 4194304 --no-cpu --no-replay --no-host > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/stats" -o c4 -- python3 bench.py --packets 4194304 --no-cpu --no-replay --no-host --steps 20 > $O/bench_prof.json 2> $O/prof.err || exit 1
timeout -k 10 600 python3 tools/pmc_traffic.py --out "$PWD/$O/pmc" --configs 1 --packets 4194304 --merge "$PWD/profiles/traffic.json" > $O/pmc.log 2>&1 || exit 1
cat $O/bench.json $O/pmc.log
