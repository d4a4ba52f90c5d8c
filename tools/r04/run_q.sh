# round 4 session 2, GPU call q: buffer loads in every shape of the plain update with no global-load path
# in the kernel (a wave whose frames span more than 4 GB sends its rows to the cold path) —
# libnfcs_prod_wbuf3 = the product — the whole GPU suite, then bench lines alternating against the previous
# product (libnfcs_prod_s2c: buffer loads in the short shape only, global-load fallback in the kernel)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4q && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4q/pytest_gpu.log 2>&1 && \
for r in 1 2 3; do for lib in prod_s2c prod_wbuf3; do
  for spec in "c1 --config 1" "c3 --config 3" "tiny --config 0 --packets 1048576" "c4 --packets 4194304" "c2 --config 2"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4q/${name}_${lib}_$r.json 2>> gpurun_out/r4q/bench.err || exit 1
  done
done; done
