"""Measurement builds (not product): load cache policies under rotation (round 5; the flow-key
kernel's header lines measured 6% faster non-temporal, profiles/r05_flowkey_load_policy_ab.jsonl):
  upd_hdrnt  the row kernels' header slot (slot 0: update, forward) non-temporal like the payload slots
  vlan_nt    every VLAN frame load non-temporal
  vlan_nt1   VLAN's slots 1.. non-temporal, slot 0 default
  vlan_wt / vlan_plain / fk_recplain   store policies (see EDITS)
Builds tools/r05/lib<variant>.so through build_lib.sh. Run here: python3 tools/r05/pol_exp.py."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
SRC = os.path.join(ROOT, "netflow_amd", "csrc")
EDITS = {
    "upd_hdrnt": [("const u32x4_t t = k == 0 ? __builtin_amdgcn_raw_buffer_load_b128(wb.rs, vo, 0, 0)",
                   "const u32x4_t t = k == 0 ? __builtin_amdgcn_raw_buffer_load_b128(wb.rs, vo, 0, kCpolNt)"),
                  ("            S.v[k] = k == 0 ? ld16<0>(a) : ld16<1>(a);",
                   "            S.v[k] = ld16<1>(a);")],
    "vlan_nt": [("        v[k] = ld16<0>((c < nl) ? src + c : zl);",
                 "        v[k] = ld16<1>((c < nl) ? src + c : zl);")],
    "vlan_nt1": [("        v[k] = ld16<0>((c < nl) ? src + c : zl);",
                  "        v[k] = k == 0 ? ld16<0>((c < nl) ? src + c : zl) : ld16<1>((c < nl) ? src + c : zl);")],
    # store policies under rotation (call u): VLAN's long-frame rows write-through / plain instead of
    # past the caches; the flow-key records plain instead of non-temporal
    "vlan_wt": [("hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_NT, 16, true>)",
                 "hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_WT, 16, true>)")],
    "vlan_plain": [("hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_NT, 16, true>)",
                    "hipLaunchKernelGGL((vlan_rows_kernel<6, 6, VST_PLAIN, 16, true>)")],
    "fk_recplain": [("            __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, (u32x4_t*)dst);",
                     "            *(u32x4_t*)dst = u32x4_t{v.x, v.y, v.z, v.w};")],
    # the update's inline checksum-byte stores (call w): the short shape write-through (c3_wt) instead
    # of past the caches; every inline store plain (c3_plain: short shape and tiny shape)
    "c3_wt": [("row_process<K, R, FWD, !FWD && R == 16 && BS == 64,", "row_process<K, R, FWD, false,")],
    "c3_plain": [("row_process<K, R, FWD, !FWD && R == 16 && BS == 64,", "row_process<K, R, FWD, false,"),
                 ("                else st8<true>(frame + pos, w >> (16 + 8 * (rl & 1u)));",
                  "                else st8<false>(frame + pos, w >> (16 + 8 * (rl & 1u)));")],
    # block orders (call x): the write passes in the read pass's XCD-aware order, so each XCD's write
    # pass reads the records and descriptors its own read pass left in its L2 (wp_xcd); flow keys in
    # dispatch order (fk_noxcd); VLAN in the XCD-aware order (vlan_xcd)
    "wp_xcd": [("__global__ __launch_bounds__(kBlock) void apply_bytes_kernel(uint8_t* __restrict__ arena,\n"
                "                                                             const nfcs_desc* __restrict__ desc,\n"
                "                                                             uint32_t n, uint32_t base16,\n"
                "                                                             const nfcs_patch* __restrict__ rec) {\n"
                "    const uint32_t lane = threadIdx.x & 63u;\n"
                "    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;",
                "__global__ __launch_bounds__(kBlock) void apply_bytes_kernel(uint8_t* __restrict__ arena,\n"
                "                                                             const nfcs_desc* __restrict__ desc,\n"
                "                                                             uint32_t n, uint32_t base16,\n"
                "                                                             const nfcs_patch* __restrict__ rec) {\n"
                "    const uint32_t lane = threadIdx.x & 63u;\n"
                "    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;"),
               ("    const uint32_t lane = threadIdx.x & 63u;\n"
                "    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;\n"
                "    const bool in = i < n;",
                "    const uint32_t lane = threadIdx.x & 63u;\n"
                "    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;\n"
                "    const bool in = i < n;")],
    "fk_noxcd": [("    const uint64_t p0 = ((uint64_t)xcd_block_n(nblocks) * kWavesPerBlock + rfl(wave)) * 64u;",
                  "    const uint64_t p0 = ((uint64_t)blockIdx.x * kWavesPerBlock + rfl(wave)) * 64u;")],
    "vlan_xcd": [("    const uint64_t pw = (uint64_t)blockIdx.x * (kBlock / R) + rfl(threadIdx.x >> 6) * PW;",
                  "    const uint64_t pw = (uint64_t)xcd_block() * (kBlock / R) + rfl(threadIdx.x >> 6) * PW;")],
    # the forward's short-mix segment stores plain (write-back) instead of past the caches (call y)
    "fwd_plain": [("                if (R == 8 && LA) st16_nt((uint4*)frame + rl, v);",
                   "                if (R == 8 && LA) st16<false>((uint4*)frame + rl, v);")],
    # the row kernels' read pass and the write passes in dispatch order instead of XCD-aware (call z)
    "rp_noxcd": [("    const uint64_t pw = (uint64_t)xcd_block_n(nblocks) * (BS / R) + rfl(threadIdx.x >> 6) * PW;",
                  "    const uint64_t pw = (uint64_t)blockIdx.x * (BS / R) + rfl(threadIdx.x >> 6) * PW;"),
                 ("    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;  // as apply_bytes_kernel",
                  "    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;  // as apply_bytes_kernel"),
                 ("    const uint64_t i = (uint64_t)xcd_block() * kBlock + threadIdx.x;\n    const nfcs_desc d",
                  "    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;\n    const nfcs_desc d")],
    # the update's short shape as the forward's short-mix rows: 8-lane rows of 12 slots, line-aligned
    # windows, 8 packets per one-wave workgroup at 6 waves/SIMD, stores write-through (c3r8) or past
    # the caches (c3r8nt) (call aa)
    "c3r8": [("        else if (shape == kShapeShort) NFCS_ROWS(7, 64, g1, SF);",
              "        else if (shape == kShapeShort) launch_rows<12, 8, 6, 64, false, SF, 1, 12>(g8, 0u, stream, arena, arena_bytes, desc, n, base16, status, patch, ws, nofwd);")],
    "c3r8nt": [("        else if (shape == kShapeShort) NFCS_ROWS(7, 64, g1, SF);",
                "        else if (shape == kShapeShort) launch_rows<12, 8, 6, 64, false, SF, 1, 12>(g8, 0u, stream, arena, arena_bytes, desc, n, base16, status, patch, ws, nofwd);"),
               ("row_process<K, R, FWD, !FWD && R == 16 && BS == 64,", "row_process<K, R, FWD, !FWD && BS == 64,")],
    # flow keys: descriptors loaded non-temporally (fk_descnt); hashes stored non-temporally (fk_hashnt)
    # (call ab)
    "fk_descnt": [("    if (p < n) dl = ((const uint2*)desc)[p];",
                   "    if (p < n) { typedef uint32_t u32x2_t __attribute__((ext_vector_type(2))); const u32x2_t t_ = __builtin_nontemporal_load((const u32x2_t*)desc + p); dl = make_uint2(t_.x, t_.y); }")],
    "fk_hashnt": [("    if (hashes && p < n) hashes[p] = hv;",
                   "    if (hashes && p < n) __builtin_nontemporal_store(hv, hashes + p);")],
    # the update's short shape in 256-thread workgroups (4 waves on one CU share the descriptor line
    # of their 16 packets through its scalar cache), buffer loads and nt stores kept (call ad)
    "c3_wg256": [("    constexpr bool BUF = !FWD && BS == 64 && R == 16;",
                  "    constexpr bool BUF = !FWD && R == 16 && (BS == 64 || !LA);"),
                 ("row_process<K, R, FWD, !FWD && R == 16 && BS == 64,", "row_process<K, R, FWD, !FWD && R == 16 && (BS == 64 || !LA),"),
                 ("        else if (shape == kShapeShort) NFCS_ROWS(7, 64, g1, SF);",
                  "        else if (shape == kShapeShort) launch_rows<6, 16, 7, kBlock, false, SF, 0, 6>(g4, 0u, stream, arena, arena_bytes, desc, n, base16, status, patch, ws, nofwd);")],
    # the forward's short-mix rows in 256-thread workgroups (call ae)
    "fwd_wg256": [("launch_rows<12, 8, 6, 64, true, SF_INLINE, 1, 12>((n + 7u) / 8u,",
                   "launch_rows<12, 8, 6, kBlock, true, SF_INLINE, 1, 12>((n + 31u) / 32u,")],
    # the tiny shapes (8-lane rows of 6 slots, 8 packets per wave) in 256-thread workgroups (call ai)
    "tiny_wg256": [("    launch_rows<6, 8, 8, 64, false, SF>(g8, 0u, stream,",
                    "    launch_rows<6, 8, 8, kBlock, false, SF>((n + 31u) / 32u, 0u, stream,"),
                   ("        launch_rows<6, 8, 8, 64, true, SF_INLINE>((n + 7u) / 8u,",
                    "        launch_rows<6, 8, 8, kBlock, true, SF_INLINE>((n + 31u) / 32u,")],
    # the forward's write pass (apply_fwd_kernel) stores write-through (sc1) / plain instead of past
    # the caches (call aj)
    "fwdwp_wt": [('    asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");',
                  '    asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");')],
    "fwdwp_plain": [('    asm volatile("global_store_short %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");',
                     '    asm volatile("global_store_short %0, %1, off" ::"v"(p), "v"(v) : "memory");')],
    # the short shape's inline byte stores with `nt` alone / `sc1 nt` instead of `sc0 sc1 nt` (call al;
    # st8_nt's other users, the forward's odd TCP offsets and VLAN's tails, see the same change)
    "c3_st_nt": [('    asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(b) : "memory");\n}\n// The same for 16 bytes',
                  '    asm volatile("global_store_byte %0, %1, off nt" ::"v"(p), "v"(b) : "memory");\n}\n// The same for 16 bytes')],
    "c3_st_sc1nt": [('    asm volatile("global_store_byte %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(b) : "memory");\n}\n// The same for 16 bytes',
                     '    asm volatile("global_store_byte %0, %1, off sc1 nt" ::"v"(p), "v"(b) : "memory");\n}\n// The same for 16 bytes')],
    # the forward's long-frame read pass with line-aligned windows in every wave (LAM 1, as the
    # update's long shape) instead of per wave (LAM 2) (call an)
    "fwd_lam1": [("launch_rows<6, 16, 7, kBlock, true, SF_DEFER, 2, 7>", "launch_rows<6, 16, 7, kBlock, true, SF_DEFER, 1, 7>")],
}

for name in sys.argv[1:] or EDITS:
    tmp = tempfile.mkdtemp()
    for f in ("nfcs_kernels.hip", "nfcs_api.hip", "nfcs_internal.h"):
        shutil.copy(os.path.join(SRC, f), tmp)
    p = os.path.join(tmp, "nfcs_kernels.hip")
    s = open(p).read()
    for a, b in EDITS[name]:
        assert s.count(a) == 1, (name, a)
        s = s.replace(a, b)
    open(p, "w").write(s)
    subprocess.run(["bash", os.path.join(ROOT, "tools/r05/build_lib.sh"), f"tools/r05/lib{name}.so"],
                   env=dict(os.environ, SRC=tmp), check=True, cwd=ROOT)
    shutil.rmtree(tmp)
    print(name, "built")
