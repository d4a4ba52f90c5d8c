# round 4 session 2, GPU call r: is the fused forward's short-mix shape (C3 mix) and the tiny shape sensitive
# to g_zero16's address as C3's short shape was? The product (g_zero16 at page offset 0x5c0) against builds
# with it at 0x900 / 0x600, alternating on one box
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4r && \
for r in 1 2 3; do for lib in prod_s2c prod_z2304 prod_z1536; do
  for spec in "fwdc3 --op l3fwd --config 3" "tiny --config 0 --packets 1048576" "vlan --op vlan"; do
    set -- $spec; name=$1; shift
    NFCS_LIB=tools/r04/libnfcs_$lib.so timeout -k 10 200 python3 -u bench.py "$@" --no-cpu --no-host --no-c4 --no-replay > gpurun_out/r4r/${name}_${lib}_$r.json 2>> gpurun_out/r4r/bench.err || exit 1
  done
done; done
