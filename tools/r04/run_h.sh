# round 4 session 2, GPU call h: the GPU suite on the product, then the product bench lines with the
# session's kernels against the session-start kernels (NFCS_LIB: libnfcs_r4_base = session start,
# libnfcs_r4_s2a = + branch-free plan and last-chunk correction, libnfcs_r4_new = + forward deferral
# above 64K packets = the product), alternating on one box; then the read-only bounds 24 / 26 (fixed)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4h && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4h/pytest_gpu.log 2>&1 && \
for r in 1 2 3; do for lib in r4_base r4_s2a r4_new; do
  for spec in "c3 --config 3" "c1 --config 1" "fwdc1 --op l3fwd --config 1" "fwdc3 --op l3fwd --config 3"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4h/${name}_${lib}_$r.json 2>> gpurun_out/r4h/bench.err || exit 1
  done
done; done && \
NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 24,26,25,27,0 --work c3 --rounds 1 --modes rotate,replay > gpurun_out/r4h/rw_c3.jsonl 2>&1 && \
NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 24,26,25,27,0 --work c1 --rounds 1 --modes rotate,replay > gpurun_out/r4h/rw_c1.jsonl 2>&1
