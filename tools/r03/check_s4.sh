#!/bin/bash
# Round 3, session 4: the whole GPU suite (the PacketBuffer mirror's new window representation goes
# through tests/test_cpp_api.py's GPU modes), smoke(), the default bench line, its kernel stats.
set -o pipefail
out=gpurun_out/${1:-r03_s4_check}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu \
   -p no:cacheprovider > $out/pytest_gpu.log 2>&1 || { tail -30 $out/pytest_gpu.log; exit 1; }
tail -1 $out/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail -20 $out/smoke.log; exit 1; }
tail -2 $out/smoke.log
timeout -k 10 400 python3 bench.py > $out/bench_default.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o c1 --output-format csv -- python3 bench.py --steps 20 --no-cpu --no-fresh --no-c4 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $out/c1_kernel_stats.csv
cut -d, -f1-4 $out/c1_kernel_stats.csv | head -5
