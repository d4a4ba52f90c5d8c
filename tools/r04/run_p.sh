# round 4 session 2, GPU call p: the product (buffer loads in the plain update's short shape): the whole GPU
# suite, smoke(), the default bench line (CPU baseline, replay / C4-shard / host sub-lines), C3, then
# rocprofv3 kernel stats of C3
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4p && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4p/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4p/smoke.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py > gpurun_out/r4p/bench_default.json 2> gpurun_out/r4p/bench_default.err && \
timeout -k 10 200 python3 -u bench.py --config 3 --no-cpu --no-host --no-c4 > gpurun_out/r4p/bench_c3.json 2> gpurun_out/r4p/bench_c3.err && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4p/prof_c3" -o c3 -- python3 bench.py --config 3 --no-cpu --no-host --no-c4 --no-replay --steps 30 > gpurun_out/r4p/prof_c3.json 2> gpurun_out/r4p/prof_c3.err
