"""CPU tests: the oracle restatement against the reference-generated golden fixtures.

tests/golden/*.{json,npz} were produced by the REFERENCE implementation (compiled from
/root/reference by tests/golden/make_golden.py); these tests pin the C restatement to it.
"""
import json
import os
import re

import numpy as np
import pytest

import oracle

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_kat():
    with open(os.path.join(GOLD, "kat.json")) as fh:
        return json.load(fh)


@pytest.mark.parametrize("name", sorted(load_kat().keys()))
def test_kat_oracle_matches_reference(oracle_lib, name):
    k = load_kat()[name]
    out, st = oracle.update_frame(bytes.fromhex(k["in"]))
    assert out.hex() == k["out"]
    assert st == k["status"]


def test_survey_appendix_b_diffs(oracle_lib):
    """The Appendix-B diff offsets (quirks Q1 TCP@l4+15, Q2 odd low byte, Q5 UDP 0->FFFF)."""
    k = load_kat()
    exp = {
        "A_main_cpp_tcp": {24: 0xE5, 25: 0x40, 49: 0xFB, 50: 0xFF},
        "B_packet_test_udp": {24: 0xF7, 25: 0x5D, 40: 0x0F, 41: 0x7E},
        "C_packet_test_tcp": {24: 0xF7, 25: 0x60, 49: 0x4B, 50: 0xED},
        "D_icmp_odd": {24: 0x7A, 25: 0xE1, 36: 0xF7, 37: 0x54},
        "E_udp_odd_ABC": {24: 0x66, 25: 0xCB, 40: 0x8F, 41: 0x50},
        "F_vlan_udp": {28: 0xF7, 29: 0x5D, 44: 0x0F, 45: 0x7E},
    }
    for name, diffs in exp.items():
        out = bytes.fromhex(k[name]["out"])
        for off, v in diffs.items():
            assert out[off] == v, (name, off)
    g = bytes.fromhex(k["G_udp_zero_to_ffff"]["out"])
    assert g[40:42] == b"\xff\xff"
    assert bytes.fromhex(k["H1_icmp_all_zero"]["out"])[36:38] == b"\xff\xff"
    assert bytes.fromhex(k["H2_icmp_sum_ffff"]["out"])[36:38] == b"\x00\x00"


def test_fuzz_oracle_matches_reference_fixture(oracle_lib):
    z = np.load(os.path.join(GOLD, "fuzz_ref.npz"))
    seed, n = int(z["seed"]), len(z["lens"])
    frames = oracle.fuzz_frames(seed, 0, n)
    arena, desc = oracle.pack_frames(frames)
    assert np.array_equal(desc["len"], z["lens"].astype(np.uint32))
    L = oracle.lib()
    h_in = np.array([L.nfo_frame_hash(oracle._ptr(arena[int(d["off16"]) * 16:]), int(d["len"]))
                     for d in desc], dtype=np.uint64)
    assert np.array_equal(h_in, z["hash_in"]), "fuzz generator drifted from the fixture"
    status, _ = oracle.update_batch(arena, desc, nthreads=4)
    assert np.array_equal(status, z["oracle_status"])
    h_out = np.array([L.nfo_frame_hash(oracle._ptr(arena[int(d["off16"]) * 16:]), int(d["len"]))
                      for d in desc], dtype=np.uint64)
    dom = (status & 0x3F) != 14
    assert np.array_equal(h_out[dom], z["hash_out"][dom])
    assert np.array_equal(h_out[~dom], h_in[~dom])  # OOB frames untouched
    # the corpus exercises every branch, including the IHL<5 overlap path
    for st in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 14, 0x42, 0x43, 0x44, 0x45):
        assert (status == st).sum() > 0, st


def test_status_codes_match_abi_header():
    hdr = open(os.path.join(ROOT, "include", "nfcs.h")).read()
    ora = open(os.path.join(ROOT, "oracle", "nfcs_oracle.h")).read()
    abi = dict((m[0], int(m[1], 0)) for m in re.findall(r"NFCS_ST_(\w+)\s*=\s*(0x[0-9a-fA-F]+|\d+)", hdr))
    orc = dict((m[0], int(m[1], 0)) for m in re.findall(r"NFO_ST_(\w+)\s*=\s*(0x[0-9a-fA-F]+|\d+)", ora))
    assert abi == orc and len(abi) == 19


def test_config_generator_and_layout(oracle_lib):
    import netflow_amd as nf
    for cfg in range(4):
        arena, desc = oracle.gen_config(cfg, 20250620, 1000, 257)
        # structural checks of the synthetic spec
        for d in desc[:16]:
            o, ln = int(d["off16"]) * 16, int(d["len"])
            f = arena[o:o + ln]
            assert f[12] == 0x08 and f[13] == 0 and f[14] == 0x45
            assert (int(f[16]) << 8 | int(f[17])) == ln - 14
            assert f[23] in (253, 6, 17)
        # the product's host layout equals the oracle's
        if os.path.exists(nf.LIB_PATH):
            d2, nb = nf.layout_config(cfg, 20250620, 1000, 257)
            assert np.array_equal(d2, desc) and nb == int(desc[-1]["off16"]) * 16 + (int(desc[-1]["len"]) + 15) // 16 * 16
    lens = oracle.layout_config(3, 20250620, 0, 20000)[0]["len"]
    assert lens.min() >= 64 and lens.max() <= 1500 and (lens % 2 == 1).sum() > 1000


def test_small_config_digest_matches_reference_golden(oracle_lib):
    """C0 (1024 x 64 B) end to end through the oracle == the reference's digest."""
    with open(os.path.join(GOLD, "configs.json")) as fh:
        g = json.load(fh)
    c0 = g["configs"]["0"]
    din, dout, hist = oracle.config_digest(0, g["seed"], 0, c0["n"], 2)
    assert f"{din:016x}" == c0["digest_in"] and f"{dout:016x}" == c0["digest_out"]
    assert hist == {1: 1024}


def test_reference_shim_cross_check():
    """Where /root/reference exists: oracle == compiled reference on fresh fuzz frames."""
    if not os.path.isdir(oracle.REFERENCE_ROOT):
        pytest.skip("reference not present (GPU box)")
    oracle.build(ref=True)
    frames = oracle.fuzz_frames(777, 0, 20000)
    for f in frames:
        o, st = oracle.update_frame(f)
        if (st & 0x3F) == 14:
            continue
        assert oracle.ref_update_frame(f) == o


def test_c4_shard_digest_matches_reference(oracle_lib):
    """BASELINE C4 (32M x 1500 B over 8 GPUs): the oracle's digest of rank 7's 4M-packet shard
    equals the reference's (configs.json c4_rank_shards, tests/golden/make_golden.py c4)."""
    import json
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "configs.json")))
    sh = g["c4_rank_shards"][7]
    assert (sh["first"], sh["n"]) == (7 << 22, 1 << 22)
    din, dout, _ = oracle.config_digest(1, 20250620, sh["first"], sh["n"], 8)
    assert (f"{din:016x}", f"{dout:016x}") == (sh["digest_in"], sh["digest_out"])


def test_oracle_under_asan_ubsan():
    """the CPU restatement built with -fsanitize=address,undefined runs every
    entry point over 200k fuzz frames held in exact-size heap buffers without a finding."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["make", "-s", "-C", here, "sanitize"], check=True)
    r = subprocess.run([os.path.join(here, "_san", "nfo_sanitize"), "200000", "9090"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "sanitize_frames=200000" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
