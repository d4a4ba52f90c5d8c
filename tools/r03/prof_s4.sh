#!/bin/bash
# Round 3, session 4: rocprofv3 kernel stats (CSV) of the C1 bench command, for profiles/.
set -o pipefail
out=gpurun_out/${1:-r03_s4_prof}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o c1 -- python3 bench.py --steps 20 --no-cpu --no-fresh --no-c4 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
find $out/prof -name "*kernel_stats.csv" > $out/files.txt
cp "$(head -1 $out/files.txt)" $out/c1_kernel_stats.csv
cut -d, -f1-5 $out/c1_kernel_stats.csv | head -6
grep -o '"frac": [0-9.]*' $out/prof.log | head -1 || true
