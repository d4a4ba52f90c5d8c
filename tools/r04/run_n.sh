# round 4 session 2, GPU call n: the product with per-wave buffer loads (lanes past a frame read zeros
# with no request): the whole GPU suite, then bench lines alternating against the session's previous
# product (libnfcs_prod_s2b: lanes past a frame load g_zero16) on one box: C3, C1, C2, the C4 shard;
# then flow keys with their zero lanes as out-of-range buffer loads (libnfcs_prod_fkbuf, timing build,
# arenas up to 4 GB) against the product
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4n && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4n/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n/smoke.log 2>&1 && \
for r in 1 2 3; do for lib in prod_s2b prod_wbuf; do
  for spec in "c3 --config 3" "c1 --config 1" "c2 --config 2" "c4 --packets 4194304" "fwdc3 --op l3fwd --config 3"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4n/${name}_${lib}_$r.json 2>> gpurun_out/r4n/bench.err || exit 1
  done
done; done && \
for r in 1 2 3; do for lib in prod_wbuf prod_fkbuf; do
  NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py --op flowkey --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4n/fk_${lib}_$r.json 2>> gpurun_out/r4n/bench.err || exit 1
done; done
