# round 4 session 2, GPU call i: C1 in one launch pair against 512K sub-batches (variant 10) under rotation,
# alternating; rocprofv3 kernel stats of the C1 line; the 8-rank path rehearsed on this one GPU
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4i && \
NFCS_LIB=tools/r04/libnfcs_r4_new.so timeout -k 10 300 python3 -u tools/r04/fresh_forms.py --torch --variants 0,10 --work c1 --rounds 4 --modes rotate,replay > gpurun_out/r4i/sub_c1.jsonl 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4i/prof_c1" -o c1 -- python3 bench.py --no-cpu --no-host --no-c4 --no-replay --steps 50 > gpurun_out/r4i/prof_c1.json 2> gpurun_out/r4i/prof_c1.err && \
NFCS_BENCH_DEVICE=0 timeout -k 10 600 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 > gpurun_out/r4i/bench_gpus8_one_box.json 2> gpurun_out/r4i/bench_gpus8.err
