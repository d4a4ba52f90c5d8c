#!/bin/bash
# Round 3: the workspace event recorded only when another stream needs it — the whole GPU suite,
# A/B against the build before (tools/exp/libnfcs_prev.so) on C1 and the C4 shard, and a kernel
# trace for the gap between back-to-back calls.
set -o pipefail
out=gpurun_out/${1:-r03_check_ws}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu \
   -p no:cacheprovider > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
for a in "c1:--config 1 --no-c4 --no-fresh" "c4shard:--packets 4194304 --no-fresh"; do
IFS=: read -r w args <<< "$a"
for r in 1 2 3; do
for lib in tools/exp/libnfcs_prev.so netflow_amd/libnfcs.so; do
  NFCS_LIB=$lib timeout -k 10 200 python3 bench.py $args --steps 20 --warmup 3 --no-cpu > $out/b.json 2> $out/b.err || { tail -5 $out/b.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$out/b.json'))
print(json.dumps({'work':'$w','lib':'$lib'.split('/')[-1],'frac':d['roofline']['frac'],'kernel_ms':d['roofline']['kernel_ms'],'ms_per_step':d['ms_per_step'],'parity':d['parity']['match']}))" | tee -a $out/ab.jsonl
done
done
done
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_c1 -o c1 -- python3 bench.py --no-cpu --no-fresh --no-c4 > $out/bench_c1_under_rocprof.json 2> $out/prof_c1.err
