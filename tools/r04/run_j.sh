# round 4 session 2, GPU call j: the GPU suite on the product (lanes past a frame load its first chunk),
# then bench C3 / C1 alternating over four libraries on one box: the product build before / after that
# change (libnfcs_prod_s2b / libnfcs_prod_zs) and the measurement builds of the same two sources
# (libnfcs_r4_new / libnfcs_r4_zs) — the product build measured 3-5% slower on C3 than the measurement
# build of the same kernel source in calls f, g and the profiling pass
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4j && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j/pytest_gpu.log 2>&1 && \
for r in 1 2 3; do for lib in prod_s2b r4_new prod_zs r4_zs; do
  for spec in "c3 --config 3" "c1 --config 1"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4j/${name}_${lib}_$r.json 2>> gpurun_out/r4j/bench.err || exit 1
  done
done; done
