# round 4, GPU call e: every bench line with the rotation (update, forward, VLAN, flow keys; C1-C3, 4M)
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4e && \
for spec in "l3fwd_c1 --op l3fwd" "l3fwd_4m --op l3fwd --packets 4194304" "l3fwd_c3 --op l3fwd --config 3" "vlan --op vlan" "flowkey --op flowkey" "flowkey_c3 --op flowkey --config 3" "c2 --config 2" "c3 --config 3" "c4shard --packets 4194304"; do
  set -- $spec; name=$1; shift
  timeout -k 10 240 python3 -u bench.py "$@" --no-cpu > gpurun_out/r4e/$name.json 2> gpurun_out/r4e/$name.err || exit 1
done
