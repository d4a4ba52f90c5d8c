"""Multi-process path of bench.py on CPU: world_size 2 over gloo (127.0.0.1); the --gpus / WORLD_SIZE
contract; the byte-balanced split of one batch (nfcs_shard_bytes).

The checksum path shards by packets with no data-path collective: each rank
owns packets [rank*n, (rank+1)*n) of the same seeded stream, and ranks only meet at the timing
barriers (max over ranks of the wall time, sum of frame bytes). This checks that harness: the
shards tile the packet stream exactly, the reductions are right, and per-shard oracle digests
add up to the digest of the whole stream (the property the N-GPU parity check relies on).
"""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws),
                      RANK=str(rank), LOCAL_RANK=str(rank), NFCS_DIST_BACKEND="gloo")
    import bench
    import oracle
    D = bench.Dist(*bench.dist_env())
    first, n = bench.shard(rank, 4096)
    D.barrier()
    mx = D.max(1.5 + rank)
    total = D.sum(float(n))
    din, dout, hist = oracle.config_digest(1, bench.SEED, first, n, 1)
    dsum = D.sum(float(dout % (1 << 40)))  # exact in float64 for 2 ranks
    dsum64 = D.sum_u64(dout)
    per = D.gather_u64(dout)  # the N > 1 line's per_gpu_digest (round 6)
    D.barrier()
    D.close()
    q.put((rank, first, n, mx, total, dout, dsum, dsum64, per))


@pytest.mark.parametrize("ws", [2])
def test_two_rank_gloo_harness(ws):
    import oracle
    oracle.build(ref=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(ws))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # shards tile [0, ws*n) exactly
    assert [(r[1], r[2]) for r in res] == [(r * 4096, 4096) for r in range(ws)]
    assert all(r[3] == 1.5 + ws - 1 for r in res)      # max over ranks
    assert all(r[4] == 4096.0 * ws for r in res)       # sum over ranks
    # digests are order-independent sums: shard digests add up to the whole stream's digest
    _, whole, _ = oracle.config_digest(1, 20250620, 0, 4096 * ws, 2)
    assert (sum(r[5] for r in res) % (1 << 64)) == whole
    assert all(r[6] == float(sum(x[5] % (1 << 40) for x in res)) for r in res)
    assert all(r[7] == whole for r in res)  # the exact u64 all-reduce
    assert all(r[8] == [x[5] for x in res] for r in res)  # the exact u64 all-gather, in rank order


def _strong_worker(rank, ws, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws),
                      RANK=str(rank), LOCAL_RANK=str(rank), NFCS_DIST_BACKEND="gloo")
    import bench
    import oracle
    D = bench.Dist(*bench.dist_env())
    first, n = bench.shard_strong(3, 1 << 22, rank, ws)  # the C3 batch, split by bytes
    import netflow_amd as nf
    desc, _ = nf.layout_config(3, bench.SEED, first, n, 128)
    nbytes = int(desc["len"].astype("i8").sum())
    _, dout, _ = oracle.config_digest(3, bench.SEED, first, n, 4)
    whole = D.sum_u64(dout)
    D.close()
    q.put((rank, first, n, nbytes, whole))


def test_two_rank_gloo_strong_split_of_c3_by_bytes():
    """ONE mixed-length batch (C3: 4M frames of U{64..1500} B) split over 2 ranks
    into contiguous ranges balanced by bytes; the ranks' byte counts are within one frame of each
    other and their (reference-pinned oracle) digests sum to the reference's digest of C3."""
    import json
    import oracle
    oracle.build(ref=False)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strong_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == 0 and res[0][1] + res[0][2] == res[1][1] and res[1][1] + res[1][2] == 1 << 22
    assert abs(res[0][3] - res[1][3]) <= 1500
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")))
    want = int(g["configs"]["3"]["digest_out"], 16)
    assert res[0][4] == res[1][4] == want


def test_gpus_flag_must_match_world_size():
    """Under a launcher WORLD_SIZE must equal --gpus: a mismatch exits non-zero before any GPU use."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--no-cpu"],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_gloo_group_log_stays_off_stdout():
    """bench.py forms its gloo group with fd 1 pointed at stderr: gloo's "[Gloo] Rank r is
    connected ..." lines go to stderr, and stdout carries only what the bench prints after."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = (
        "import os, sys; sys.path.insert(0, %r); import bench\n"
        "with bench.stdout_to_stderr():\n"
        "    os.write(1, b'[Gloo] native write\\n'); print('python print', flush=True)\n"
        "print('{\"line\": 1}')\n" % root)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip().splitlines() == ['{"line": 1}']
    assert "[Gloo] native write" in r.stderr and "python print" in r.stderr


def _solo_worker(rank, ws, port, q):
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(ws),
                      RANK=str(rank), LOCAL_RANK=str(rank), NFCS_DIST_BACKEND="gloo")
    import bench
    D = bench.Dist(*bench.dist_env())
    log = []

    def timed(pre=None):  # a rank's "steps": sleeps, stamped
        t0 = time.time()
        if pre is not None:
            pre()
        time.sleep(0.05 + 0.02 * rank)
        log.append((t0, time.time(), pre is not None))
        return time.time() - t0

    solo, t_rank, wall = bench.scaling_timings(D, timed, 2e9, 10, True, pre=lambda: None,
                                               after=lambda: log.append(("after", time.time())))
    D.close()
    q.put((rank, solo, t_rank, wall, log))


def test_two_rank_solo_shard_then_concurrent_region():
    """bench.py's N > 1 timing (bench.scaling_timings) over gloo, 2 ranks on CPU:
    rank 0 times its shard ALONE first (rank 1 runs nothing until rank 0 is done), every rank gets
    rank 0's solo rate, then both time the concurrent region; the line's wall time is the max over
    ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_solo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, solo0, t0r, wall0, log0), (_, solo1, t1r, wall1, log1) = res
    solo_run = [e for e in log0 if len(e) == 3 and e[2]]
    assert len(solo_run) == 1 and not any(len(e) == 3 and e[2] for e in log1)  # only rank 0 ran solo
    conc1 = [e for e in log1 if len(e) == 3][0]
    assert conc1[0] >= solo_run[0][1] - 1e-3  # rank 1 started after rank 0's solo region ended
    want = 2e9 / ((solo_run[0][1] - solo_run[0][0]) / 10) / 1e9
    assert solo0 == solo1 and abs(solo0 - want) / want < 0.2
    assert wall0 == wall1 == max(t0r, t1r)
    assert any(e[0] == "after" for e in log0) and any(e[0] == "after" for e in log1)
