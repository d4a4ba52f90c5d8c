# round 4, GPU call d: short-shape slot counts on C3, then the round-4 profiles of every line
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/r4d && \
timeout -k 10 200 python3 -u tools/r04/fresh_forms.py --variants 0,17,18,19 --work c3 --rounds 2 --modes rotate > gpurun_out/r4d/slots_c3.jsonl 2>&1 && \
bash tools/r04/prof_all.sh r4d/prof
