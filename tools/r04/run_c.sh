# round 4, GPU call c: the software-pipelined short shape on C3
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4c && \
timeout -k 10 300 python3 -u tools/r04/fresh_forms.py --variants 0,15,50,51,52,53,54,55,56,57 --work c3 --rounds 2 --modes rotate > gpurun_out/r4c/pipe_c3.jsonl 2>&1
