# round 4 session 2, GPU call o: buffer loads only in the plain update's one-wave shapes (short: C3; tiny:
# 1M x 64-byte frames in 128-byte slots) — libnfcs_prod_wbuf2 — against libnfcs_prod_s2b, alternating on one
# box; C1, the C4 shard and the forward's C3 mix should be unchanged (they keep global loads)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4o && \
for r in 1 2 3; do for lib in prod_s2b prod_wbuf2; do
  for spec in "c3 --config 3" "tiny --config 0 --packets 1048576" "c1 --config 1" "c4 --packets 4194304" "fwdc3 --op l3fwd --config 3"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4o/${name}_${lib}_$r.json 2>> gpurun_out/r4o/bench.err || exit 1
  done
done; done
