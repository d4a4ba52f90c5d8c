# round 4, GPU call b: 64-byte-record deferral forms (C1, C3, C4 shard), then the bench default line
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4b && \
timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,1,30,31,32,40,41,42 --work c1 --rounds 2 > gpurun_out/r4b/forms_c1.jsonl 2>&1 && \
timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,15,33,34,14 --work c3 --rounds 2 > gpurun_out/r4b/forms_c3.jsonl 2>&1 && \
timeout -k 10 240 python3 -u tools/r04/fresh_forms.py --variants 0,30,31 --work c4shard --rounds 1 > gpurun_out/r4b/forms_c4.jsonl 2>&1 && \
timeout -k 10 300 python3 -u bench.py > gpurun_out/r4b/bench.json 2> gpurun_out/r4b/bench.err && \
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4b/pytest.log 2>&1
