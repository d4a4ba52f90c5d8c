"""The C++ host API (include/netflow_amd/packet.hpp): compiled with g++ against the C ABI,
PacketBuffer/Packet semantics on CPU, bit-exact batched and single-packet updates on GPU."""
import json
import os
import subprocess

import pytest

import netflow_amd as nf
import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "packet_shim_test.cpp")
EXE = os.path.join(ROOT, "tests", "cpp", "packet_shim_test")


@pytest.fixture(scope="module")
def exe():
    if not os.path.exists(nf.LIB_PATH):
        nf.build()
    libdir = os.path.dirname(nf.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"), SRC,
                    "-o", EXE, "-L" + libdir, "-l:" + os.path.basename(nf.LIB_PATH),
                    "-Wl,-rpath," + libdir, "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return EXE


def test_cpp_api_semantics_cpu(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True)
    assert "api_failures=0" in r.stdout, r.stdout + r.stderr
    if not os.path.exists("/dev/kfd"):
        assert "engine_without_gpu_throws=1" in r.stdout  # no silent CPU fallback


def _frames():
    kat = json.load(open(os.path.join(ROOT, "tests", "golden", "kat.json")))
    names = sorted(kat)
    frames = [bytes.fromhex(kat[k]["in"]) for k in names] + oracle.fuzz_frames(31337, 0, 3000)
    return frames


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["batch", "single"])
def test_cpp_update_matches_oracle(exe, mode):
    frames = _frames() if mode == "batch" else _frames()[:200]
    r = subprocess.run([exe, mode], input="\n".join(f.hex() for f in frames) + "\n",
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    assert len(lines) == len(frames)
    for f, line in zip(frames, lines):
        st, hx = (line.split(" ") + [""])[:2]
        exp, est = oracle.update_frame(f)
        if (est & 0x3F) == 14:  # outside the parity domain: untouched
            assert hx == f.hex()
            continue
        assert hx == exp.hex()
        if mode == "batch":
            assert int(st) == est
