"""The checksum path over NIC-ring slot strides: frames laid out at the starts of
2048-byte slots (a power-of-two mbuf data room) and of 2176-byte slots (2048 + 128 bytes of
headroom, netflow_amd::BufferPool's default), and the BASELINE configs' own 128-byte alignment.
Every layout must give the reference's bytes: whole-arena digests against the compiled reference's
(tests/golden/configs.json) for C1 (1M x 1500 B), the C4 shard (4M x 1500 B, sub-batched, every wave
deferred) and the C3 mix (4M x U{64..1500} B), and the fused forward's 4M x 1500 B digest."""
import json
import os

import numpy as np
import pytest

import netflow_amd as nf

pytestmark = pytest.mark.gpu
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "configs.json")))
SEED = 20250620


def want(config, n):
    c = GOLD["configs"].get(str(config))
    if c and c["first"] == 0 and c["n"] == n:
        return c["digest_out"]
    for sh in GOLD.get("c4_rank_shards", []):
        if config == 1 and sh["first"] == 0 and sh["n"] == n:
            return sh["digest_out"]
    raise KeyError((config, n))


@pytest.mark.parametrize("stride", [2048, 2176])
@pytest.mark.parametrize("config,n", [(1, 1 << 20), (1, 1 << 22), (3, 1 << 22)])
def test_update_at_slot_stride_matches_reference(engine, stride, config, n):
    d_arena, nbytes, d_desc, hdesc = engine.config_batch(config, SEED, 0, n, stride)
    try:
        assert int(hdesc["off16"][1]) * 16 == stride  # one frame per slot
        engine.update_device(d_arena, nbytes, d_desc, n)
        engine.sync()
        assert f"{engine.digest_device(d_arena, nbytes, d_desc, n, 0):016x}" == want(config, n)
    finally:
        d_arena.free()
        d_desc.free()


@pytest.mark.parametrize("stride", [2048, 2176])
def test_l3_forward_4m_at_slot_stride_matches_reference(engine, stride):
    g = [x for x in GOLD["l3fwd_more"] if x["config"] == 1 and x["first"] == 0 and x["n"] == 1 << 22]
    assert g, "l3fwd_more holds the 4M x 1500 B forward digest"
    n = 1 << 22
    table = np.frombuffer(bytes.fromhex(GOLD["l3fwd_c1"]["table"]), dtype=np.uint8).copy()
    d_arena, nbytes, d_desc, _ = engine.config_batch(1, SEED, 0, n, stride)
    d_tab = engine.alloc(table.nbytes).upload(table)
    d_nh = engine.alloc(4 * n).upload((np.arange(n) % 9).astype(np.uint32))
    try:
        engine.l3_forward_device(d_arena, nbytes, d_desc, d_nh, n, d_tab, 8)
        engine.sync()
        assert f"{engine.digest_device(d_arena, nbytes, d_desc, n, 0):016x}" == g[0]["digest_out"]
    finally:
        for b in (d_arena, d_desc, d_tab, d_nh):
            b.free()
