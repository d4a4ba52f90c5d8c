#!/bin/bash
# Round 3: the update at NIC-ring slot strides + the box's CPU allotment.
set -o pipefail
out=${1:-gpurun_out/r03_stride}
mkdir -p "$out"
{ echo "nproc=$(nproc)"; python3 -c 'import os; print("affinity", len(os.sched_getaffinity(0)), "cpu_count", os.cpu_count())';
  cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo "no cgroup v2 cpu.max"; 
  ls /sys/devices/system/node/ | grep node; lscpu | head -30; } > "$out/sysinfo.txt" 2>&1
for a in 128 2048 2176 1536; do
  timeout -k 10 150 python3 bench.py --no-cpu --no-fresh --steps 20 --align $a > "$out/c1_a$a.json" || exit 1
  timeout -k 10 150 python3 bench.py --no-cpu --no-fresh --steps 10 --packets 4194304 --align $a > "$out/c4_a$a.json" || exit 1
done
