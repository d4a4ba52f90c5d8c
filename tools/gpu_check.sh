#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; a crash/timeout/abort ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-run}
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures, not a fault

timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -5 "$OUT/pytest_gpu.log"; ok $rc || exit $rc

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 "$OUT/smoke.log"; ok $rc || exit $rc

for cfg in 1 2 3; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu > "$OUT/bench_c$cfg.json" 2> "$OUT/bench_c$cfg.err"
  rc=$?; echo "bench c$cfg rc=$rc"; cat "$OUT/bench_c$cfg.json"; [ $rc -eq 0 ] || exit $rc
done

for op in l3fwd flowkey vlan; do
  timeout -k 10 300 python bench.py --op $op --steps 20 --warmup 3 --no-cpu > "$OUT/bench_$op.json" 2> "$OUT/bench_$op.err"
  rc=$?; echo "bench $op rc=$rc"; cat "$OUT/bench_$op.json"; [ $rc -eq 0 ] || exit $rc
done

export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o c1 -- \
  python3 bench.py --config 1 --steps 20 --warmup 3 --no-cpu > "$OUT/prof_c1.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 "$OUT/prof_c1.log"
exit $rc
