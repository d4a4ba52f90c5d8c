"""netflow_amd — MI355X-native batched Internet-checksum engine for NetFlow++'s
``Packet::update_checksums()`` path (include/netflow++/packet.hpp:722-912).

The compute lives in ``libnfcs.so`` (hand-written gfx950 HIP kernels behind the C ABI in
``include/nfcs.h``). This module is a thin ctypes host layer over that ABI: device buffers,
contexts, the batched update on device-resident or host-resident frames, synthetic batches
and digests. It never computes a checksum itself and has no CPU fallback: if the HIP
library is missing or no gfx950 device is present, it raises.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("NFCS_LIB") or os.path.join(HERE, "libnfcs.so")
HEADER = os.path.join(ROOT, "include", "nfcs.h")
SOURCES = [os.path.join(HERE, "csrc", "nfcs_kernels.hip"), os.path.join(HERE, "csrc", "nfcs_api.hip")]

DESC_DTYPE = np.dtype([("off16", "<u4"), ("len", "<u4")])
PATCH_DTYPE = np.dtype([("ip_off", "<u2"), ("l4_off", "<u2"), ("ip", "u1", (2,)), ("l4", "u1", (2,))])

# status codes (include/nfcs.h)
ST_NONE, ST_V4, ST_V4_TCP, ST_V4_UDP, ST_V4_ICMP, ST_V4_L4SKIP = 0, 1, 2, 3, 4, 5
ST_V6, ST_V6_TCP, ST_V6_UDP, ST_V6_L4SKIP, ST_OOB, ST_BAD_DESC = 6, 7, 8, 9, 14, 15
ST_FLAG_OVERLAP = 0x40
ST_NO_ROUTE, ST_NOT_IPV4, ST_TTL_EXPIRED, ST_FLAG_FWD = 11, 12, 13, 0x80
NH_NONE = 0xFFFFFFFF
ST_VLAN_FAIL, ST_FLAG_VLAN = 16, 0x20
VLAN_NOP, VLAN_PUSH, VLAN_POP = 0, 0x40000000, 0x80000000


def vlan_push_op(vid: int, prio: int = 0) -> int:
    """NFCS_VLAN_PUSH_OP(vid, prio): the edit word of Packet::push_vlan(vid, prio)."""
    return VLAN_PUSH | ((prio & 7) << 13) | (vid & 0xFFF)

NEXTHOP_DTYPE = np.dtype([("dst_mac", "u1", (6,)), ("src_mac", "u1", (6,))])
FLOW_KEY_DTYPE = np.dtype([("hash", "<u4"), ("vlan_id", "<u2"), ("ethertype", "<u2"),
                           ("src_mac", "u1", (6,)), ("dst_mac", "u1", (6,)), ("protocol", "u1"),
                           ("is_ipv6", "u1"), ("src_port", "<u2"), ("dst_port", "<u2"),
                           ("reserved", "u1", (6,)), ("src_ip", "u1", (16,)), ("dst_ip", "u1", (16,))])
assert FLOW_KEY_DTYPE.itemsize == 64
CFG_C0, CFG_C1, CFG_C2, CFG_C3 = 0, 1, 2, 3
HOST_PATCH_ONLY, HOST_ZERO_COPY, HOST_FRAMES = 1, 2, 4
PATCH_NONE = 0xFFFF


class NfcsError(RuntimeError):
    pass


# The first 8 kernel arguments go into SGPRs at dispatch (gfx950 kernarg preloading): the row
# kernel orders its arguments so that everything a wave reads before its frame loads is among them
# (nfcs_kernels.hip, update_rows_kernel). Round 3 A/B on one box: C3 +0.5-0.8%, 1M x 64 B +1.7%,
# flow keys +1%, C1 / C2 / the fused forward / VLAN within +-0.5% (profiles/r03_s1_ab_kernarg_preload.jsonl).
KERNARG_PRELOAD = ["-mllvm", "-amdgpu-kernarg-preload-count=8"]


def build(verbose: bool = False) -> str:
    """Compile the gfx950 kernels + C ABI into netflow_amd/libnfcs.so (in-tree). The measurement
    build (extra launch forms for A/B runs) is separate: tools/r04/build.sh."""
    out = os.path.join(HERE, "libnfcs.so")
    cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", *KERNARG_PRELOAD,
           "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(HERE, "csrc"), *SOURCES, "-o", out]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    return out


# include/nfcs.h NFCS_ABI_VERSION: 2 = nfcs_update_host_frames, descriptors in any order for
# nfcs_update_host
ABI_VERSION = 2
_lib = None
_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64


def _declare(L):
    sig = {
        "nfcs_abi_version": ([], ctypes.c_int),
        "nfcs_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "nfcs_last_hip_error": ([], ctypes.c_int),
        "nfcs_ctx_create": ([ctypes.c_int, ctypes.POINTER(_vp)], ctypes.c_int),
        "nfcs_ctx_destroy": ([_vp], ctypes.c_int),
        "nfcs_ctx_stream": ([_vp], _vp),
        "nfcs_ctx_set_slot_bytes": ([_vp, ctypes.c_uint32], ctypes.c_int),
        "nfcs_ctx_launch_footprint": ([_vp, _u64, _vp, _u32, ctypes.POINTER(_u64)], ctypes.c_int),
        "nfcs_update_device": ([_vp, _vp, _u64, _vp, _u32, _vp, _vp, _vp], ctypes.c_int),
        "nfcs_update_host": ([_vp, _vp, _u64, _vp, _u32, _vp, _u32], ctypes.c_int),
        "nfcs_update_host_frames": ([_vp, _vp, _vp, _u32, _vp, _u32], ctypes.c_int),
        "nfcs_layout_config": ([ctypes.c_int, _u64, _u64, _u32, _u32, _vp, ctypes.POINTER(_u64)], ctypes.c_int),
        "nfcs_shard_bytes": ([_vp, _u32, _u32, _vp], ctypes.c_int),
        "nfcs_ctx_host_numa": ([_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        "nfcs_gen_config_device": ([_vp, ctypes.c_int, _u64, _u64, _u32, _vp, _u64, _vp, _vp], ctypes.c_int),
        "nfcs_digest_device": ([_vp, _vp, _u64, _vp, _u32, _u64, ctypes.POINTER(_u64), _vp], ctypes.c_int),
        "nfcs_device_alloc": ([_vp, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
        "nfcs_device_free": ([_vp, _vp], ctypes.c_int),
        "nfcs_host_alloc": ([_vp, ctypes.c_size_t, ctypes.POINTER(_vp)], ctypes.c_int),
        "nfcs_host_free": ([_vp, _vp], ctypes.c_int),
        "nfcs_memcpy_h2d": ([_vp, _vp, _vp, ctypes.c_size_t], ctypes.c_int),
        "nfcs_memcpy_d2h": ([_vp, _vp, _vp, ctypes.c_size_t], ctypes.c_int),
        "nfcs_stream_sync": ([_vp, _vp], ctypes.c_int),
        "nfcs_time_update_device": ([_vp, _vp, _u64, _vp, _u32, _vp, ctypes.c_int, _vp,
                                     ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "nfcs_time_update_batches": ([_vp, _u32, _vp, _vp, _vp, _u32, ctypes.c_int, _vp,
                                      ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "nfcs_l3_forward_device": ([_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u32, _vp, _vp],
                                   ctypes.c_int),
        "nfcs_vlan_device": ([_vp, _vp, _u64, _vp, _u32, _vp, _u32, _vp, _u32, _vp, _vp],
                             ctypes.c_int),
        "nfcs_time_vlan_device": ([_vp, _vp, _u64, _vp, _u32, _u32, _u32, _u32, _vp, ctypes.c_int,
                                   _vp, ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "nfcs_flow_keys_device": ([_vp, _vp, _u64, _vp, _u32, _vp, _vp, _vp], ctypes.c_int),
        "nfcs_time_stream_read": ([_vp, _vp, _u64, ctypes.c_int, ctypes.c_int, _vp, _vp], ctypes.c_int),
        "nfcs_time_frames_read": ([_vp, _vp, _u64, _vp, _u32, ctypes.c_int, _vp, _vp], ctypes.c_int),
        "nfcs_time_flow_keys_device": ([_vp, _vp, _u64, _vp, _u32, _vp, _vp, ctypes.c_int, _vp,
                                        ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
        "nfcs_time_l3_forward_device": ([_vp, _vp, _u64, _vp, _vp, _u32, _vp, _u32, _vp,
                                         ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_float)],
                                        ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        # a measurement build of an earlier round (NFCS_LIB, A/B runs) may lack a later entry point;
        # the product library exports every one (tests/test_abi.py)
        if os.environ.get("NFCS_LIB") and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


def lib() -> ctypes.CDLL:
    """Load libnfcs.so. Raises if the HIP library has not been built: there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NfcsError(f"{LIB_PATH} is missing: build it with netflow_amd.build() "
                            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
        _lib = _declare(ctypes.CDLL(LIB_PATH))
        v = _lib.nfcs_abi_version()
        # a measurement build of an earlier round (NFCS_LIB) may carry an older ABI
        if v != ABI_VERSION and not (os.environ.get("NFCS_LIB") and 1 <= v < ABI_VERSION):
            raise NfcsError(f"libnfcs.so ABI {v}, this package needs {ABI_VERSION}")
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        L = lib()
        raise NfcsError(f"{what}: {L.nfcs_strerror(rc).decode()} (rc={rc}, hip={L.nfcs_last_hip_error()})")


def layout_config(config: int, seed: int, first: int, n: int, align: int = 16):
    """Descriptors of n synthetic frames of `config` (`align`-byte aligned, arena order)."""
    desc = np.zeros(n, dtype=DESC_DTYPE)
    nbytes = _u64()
    _check(lib().nfcs_layout_config(config, seed, first, n, align, desc.ctypes.data if n else None,
                                    ctypes.byref(nbytes)), "nfcs_layout_config")
    return desc, int(nbytes.value)


def shard_bytes(desc: np.ndarray, parts: int) -> np.ndarray:
    """nfcs_shard_bytes: parts + 1 packet bounds; part p = packets [b[p], b[p+1]), its frame bytes
    within one frame of total / parts (multi-GPU partition)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    bounds = np.zeros(parts + 1, dtype=np.uint32)
    _check(lib().nfcs_shard_bytes(desc.ctypes.data if len(desc) else None, len(desc), parts,
                                  bounds.ctypes.data), "nfcs_shard_bytes")
    return bounds


class DeviceBuffer:
    """A raw device allocation owned by an Engine (no torch types involved)."""

    def __init__(self, engine: "Engine", nbytes: int):
        self.engine = engine
        self.nbytes = int(nbytes)
        p = _vp()
        _check(lib().nfcs_device_alloc(engine.ctx, max(self.nbytes, 16), ctypes.byref(p)), "device_alloc")
        self.ptr = p.value

    def upload(self, a: np.ndarray, offset: int = 0):
        """Copy `a` into the buffer at byte `offset`."""
        a = np.ascontiguousarray(a)
        if offset < 0 or offset + a.nbytes > self.nbytes:
            raise NfcsError(f"upload of {a.nbytes} B at {offset} past a {self.nbytes}-byte buffer")
        if a.nbytes:
            _check(lib().nfcs_memcpy_h2d(self.engine.ctx, self.ptr + offset, a.ctypes.data, a.nbytes), "h2d")
        return self

    def download(self, dtype=np.uint8, count: int | None = None, offset: int = 0) -> np.ndarray:
        """`count` items of `dtype` from byte `offset` (default: the rest of the buffer)."""
        dtype = np.dtype(dtype)
        count = (self.nbytes - offset) // dtype.itemsize if count is None else count
        if offset < 0 or offset + count * dtype.itemsize > self.nbytes:
            raise NfcsError(f"download of {count} x {dtype} at {offset} past a {self.nbytes}-byte buffer")
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            _check(lib().nfcs_memcpy_d2h(self.engine.ctx, out.ctypes.data, self.ptr + offset, out.nbytes), "d2h")
        return out

    def free(self):
        if self.ptr:
            lib().nfcs_device_free(self.engine.ctx, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Engine:
    """One nfcs context on one device (nfcs_ctx_create)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._pinned = {}  # address -> size of the host_array() allocations still held
        c = _vp()
        _check(lib().nfcs_ctx_create(device, ctypes.byref(c)), f"nfcs_ctx_create({device})")
        self.ctx = c.value

    def close(self):
        if getattr(self, "ctx", None):
            for p in list(self._pinned):
                lib().nfcs_host_free(self.ctx, p)
            self._pinned.clear()
            lib().nfcs_ctx_destroy(self.ctx)
            self.ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def stream(self) -> int:
        return lib().nfcs_ctx_stream(self.ctx)

    def set_slot_bytes(self, nbytes: int):
        """Launch-shape hint for the device-path calls that follow (nfcs_ctx_set_slot_bytes): the
        mean arena bytes per frame of bursts that fill only part of their arena; 0 = arena_bytes / n."""
        _check(lib().nfcs_ctx_set_slot_bytes(self.ctx, int(nbytes)), "set_slot_bytes")

    def launch_footprint(self, arena_bytes: int, desc, n: int) -> int:
        """The mean footprint per packet the next device call over this burst picks its launch
        shape from (nfcs_ctx_launch_footprint; speed only)."""
        m = _u64()
        p = desc.ptr if isinstance(desc, DeviceBuffer) else int(desc)
        _check(lib().nfcs_ctx_launch_footprint(self.ctx, arena_bytes, p, n, ctypes.byref(m)), "launch_footprint")
        return int(m.value)

    def host_numa(self) -> tuple[int, bool]:
        """(NUMA node of this GPU or -1, whether the host staging ring is bound to it)."""
        node, local = ctypes.c_int(), ctypes.c_int()
        _check(lib().nfcs_ctx_host_numa(self.ctx, ctypes.byref(node), ctypes.byref(local)), "host_numa")
        return node.value, bool(local.value)

    def alloc(self, nbytes: int) -> DeviceBuffer:
        return DeviceBuffer(self, nbytes)

    def host_array(self, nbytes: int) -> np.ndarray:
        """A pinned host uint8 array (nfcs_host_alloc). Release it with host_free(); whatever is
        still held when the engine closes is freed then (do not use such arrays afterwards)."""
        p = _vp()
        size = max(int(nbytes), 16)
        _check(lib().nfcs_host_alloc(self.ctx, size, ctypes.byref(p)), "host_alloc")
        self._pinned[p.value] = size
        return np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p.value))[:nbytes]

    def host_free(self, arr: np.ndarray):
        """Free a host_array() allocation now (the array must not be used afterwards)."""
        p = arr.__array_interface__["data"][0]
        if self._pinned.pop(p, None) is None:
            raise NfcsError("host_free: not a live host_array of this engine")
        _check(lib().nfcs_host_free(self.ctx, p), "host_free")

    def sync(self, stream=None):
        _check(lib().nfcs_stream_sync(self.ctx, stream), "stream_sync")

    # ---- the hot path -------------------------------------------------------------------
    def update_device(self, arena: DeviceBuffer | int, arena_bytes: int, desc: DeviceBuffer | int,
                      n: int, status=None, patch=None, stream=None):
        """Batched update_checksums() on device-resident frames (async on `stream`)."""
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_update_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), n,
                                        ptr(status), ptr(patch), stream), "nfcs_update_device")

    def update_host(self, arena: np.ndarray, desc: np.ndarray, want_status: bool = True,
                    mode: str = "patch") -> np.ndarray | None:
        """Batched update_checksums() on host frames (in place); returns status bytes.
        mode: "patch" (default: frames H2D, patch records back), "frames" (whole frames back),
        "zero_copy" (pinned arena from host_array(): the kernel reads it over PCIe in place)."""
        flags = {"patch": 0, "frames": HOST_FRAMES, "zero_copy": HOST_ZERO_COPY}[mode]
        assert arena.dtype == np.uint8 and arena.flags.c_contiguous
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        n = len(desc)
        status = np.zeros(n, dtype=np.uint8) if want_status else None
        _check(lib().nfcs_update_host(self.ctx, arena.ctypes.data, arena.nbytes,
                                      desc.ctypes.data if n else None, n,
                                      status.ctypes.data if want_status and n else None,
                                      flags), "nfcs_update_host")
        return status

    def update_host_frames(self, buf: np.ndarray, offsets: np.ndarray, lens: np.ndarray,
                           want_status: bool = True) -> np.ndarray | None:
        """Batched update_checksums() on n frames scattered in host memory (nfcs_update_host_frames):
        frame i is buf[offsets[i] : offsets[i] + lens[i]] (any byte offset, any order; offsets[i] < 0
        passes a NULL frame), updated in place; returns status bytes."""
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        offsets = np.asarray(offsets, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        n = len(lens)
        assert len(offsets) == n and (n == 0 or int((offsets + lens.astype(np.int64)).max()) <= buf.nbytes)
        ptrs = np.where(offsets < 0, 0, np.uint64(buf.ctypes.data) + offsets.astype(np.uint64)).astype(np.uint64)
        status = np.zeros(n, dtype=np.uint8) if want_status else None
        _check(lib().nfcs_update_host_frames(self.ctx, ptrs.ctypes.data if n else None,
                                             lens.ctypes.data if n else None, n,
                                             status.ctypes.data if want_status and n else None, 0),
               "nfcs_update_host_frames")
        return status

    def l3_forward_device(self, arena, arena_bytes: int, desc, nh, n: int, table, table_n: int,
                          status=None, stream=None):
        """Fused transit-IPv4 forward (TTL--, MAC rewrite, update_checksums) on device frames;
        nh = n u32 next-hop indexes, table = table_n nfcs_nexthop records (12 bytes each)."""
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_l3_forward_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), ptr(nh), n,
                                            ptr(table), table_n, ptr(status), stream),
               "nfcs_l3_forward_device")

    def vlan_device(self, arena, arena_bytes: int, desc, n: int, ops=None, op_all: int = 0,
                    caps=None, cap_all: int = 0, status=None, stream=None):
        """Batched Packet::push_vlan / pop_vlan + update_checksums on device frames; desc
        lengths are updated in place. ops: n u32 edit words (or op_all for every packet),
        caps: n u32 buffer capacities from the frame start (or cap_all)."""
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_vlan_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), n, ptr(ops),
                                      op_all, ptr(caps), cap_all, ptr(status), stream),
               "nfcs_vlan_device")

    def time_vlan_device(self, arena, arena_bytes, desc, n, op_all, op_alt, cap_all, iters,
                         status=None, stream=None) -> float:
        ms = ctypes.c_float()
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_time_vlan_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), n, op_all,
                                           op_alt, cap_all, ptr(status), iters, stream,
                                           ctypes.byref(ms)), "time_vlan_device")
        return float(ms.value)

    def flow_keys_device(self, arena, arena_bytes: int, desc, n: int, keys=None, hashes=None,
                         stream=None):
        """PacketClassifier::extract_flow_key + hash_flow on device frames: n 64-byte
        FLOW_KEY_DTYPE records and/or n u32 hashes."""
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_flow_keys_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), n, ptr(keys),
                                           ptr(hashes), stream), "nfcs_flow_keys_device")

    def time_flow_keys_device(self, arena, arena_bytes, desc, n, keys, hashes, iters,
                              stream=None) -> float:
        ms = ctypes.c_float()
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_time_flow_keys_device(self.ctx, ptr(arena), arena_bytes, ptr(desc), n,
                                                ptr(keys), ptr(hashes), iters, stream,
                                                ctypes.byref(ms)), "time_flow_keys_device")
        return float(ms.value)

    def time_stream_read(self, buf, nbytes, iters, form=0, stream=None) -> float:
        """Total ms of `iters` pure reads of buf's first nbytes (nfcs_time_stream_read): the
        read-stream reference the bench reports its kernels against."""
        ms = ctypes.c_float()
        p = buf.ptr if isinstance(buf, DeviceBuffer) else int(buf)
        _check(lib().nfcs_time_stream_read(self.ctx, p, nbytes & ~15, form, iters, stream,
                                           ctypes.byref(ms)), "time_stream_read")
        return float(ms.value)

    def time_frames_read(self, arena, arena_bytes, desc, n, iters, stream=None) -> float:
        """Total ms of `iters` reads of the batch's frames in the checksum read pass's own access
        pattern, nothing computed or written (nfcs_time_frames_read)."""
        ms = ctypes.c_float()
        p = lambda b: b.ptr if isinstance(b, DeviceBuffer) else int(b)
        _check(lib().nfcs_time_frames_read(self.ctx, p(arena), arena_bytes, p(desc), n, iters, stream,
                                           ctypes.byref(ms)), "time_frames_read")
        return float(ms.value)

    def time_l3_forward_device(self, arena, arena_bytes, desc, nh, n, table, table_n, iters,
                               status=None, stream=None) -> float:
        ms = ctypes.c_float()
        ptr = lambda b: None if b is None else (b.ptr if isinstance(b, DeviceBuffer) else int(b))
        _check(lib().nfcs_time_l3_forward_device(self.ctx, ptr(arena), arena_bytes, ptr(desc),
                                                 ptr(nh), n, ptr(table), table_n, ptr(status),
                                                 iters, stream, ctypes.byref(ms)),
               "time_l3_forward_device")
        return float(ms.value)

    def time_update_device(self, arena, arena_bytes, desc, n, iters, status=None, stream=None) -> float:
        ms = ctypes.c_float()
        _check(lib().nfcs_time_update_device(self.ctx, arena.ptr, arena_bytes, desc.ptr, n,
                                             None if status is None else status.ptr, iters, stream,
                                             ctypes.byref(ms)), "time_update_device")
        return float(ms.value)

    def time_update_batches(self, batches, n, iters, stream=None) -> float:
        """Total ms of `iters` back-to-back update_device calls rotating over `batches` — a list of
        (arena, arena_bytes, desc), n packets each — on one stream (nfcs_time_update_batches): the
        steady state of a NIC ring, where no call re-processes what the previous one wrote."""
        k = len(batches)
        p = lambda b: b.ptr if isinstance(b, DeviceBuffer) else int(b)
        arenas = (_vp * k)(*[p(a) for a, _, _ in batches])
        sizes = (_u64 * k)(*[int(nb) for _, nb, _ in batches])
        descs = (_vp * k)(*[p(d) for _, _, d in batches])
        ms = ctypes.c_float()
        _check(lib().nfcs_time_update_batches(self.ctx, k, arenas, sizes, descs, n, iters, stream,
                                              ctypes.byref(ms)), "time_update_batches")
        return float(ms.value)

    # ---- synthetic batches / digests ----------------------------------------------------
    def gen_config_device(self, config: int, seed: int, first: int, n: int,
                          arena: DeviceBuffer, arena_bytes: int, desc: DeviceBuffer, stream=None):
        _check(lib().nfcs_gen_config_device(self.ctx, config, seed, first, n, arena.ptr, arena_bytes,
                                            desc.ptr, stream), "gen_config_device")

    def digest_device(self, arena: DeviceBuffer, arena_bytes: int, desc: DeviceBuffer, n: int,
                      first: int = 0, stream=None) -> int:
        out = _u64()
        _check(lib().nfcs_digest_device(self.ctx, arena.ptr, arena_bytes, desc.ptr, n, first,
                                        ctypes.byref(out), stream), "digest_device")
        return int(out.value)

    def config_batch(self, config: int, seed: int, first: int, n: int, align: int = 16):
        """Lay out + generate a synthetic batch on the device. Returns (arena, nbytes, desc, host_desc)."""
        hdesc, nbytes = layout_config(config, seed, first, n, align)
        d_desc = self.alloc(max(hdesc.nbytes, 16)).upload(hdesc)
        d_arena = self.alloc(max(nbytes, 16))
        self.gen_config_device(config, seed, first, n, d_arena, nbytes, d_desc)
        self.sync()
        return d_arena, nbytes, d_desc, hdesc
