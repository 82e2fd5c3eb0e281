"""Codegen guards for the LDS-DMA batch kernel (CPU: hipcc cross-compiles gfx950).

Two silent performance cliffs were hit while developing the LDS-DMA batch kernel
(kopia_amd/csrc/kcdc_kernels.hip) and are pinned here:
* a runtime flag tested inside the tile loop made hipcc treat the tile state as
  divergent: every LDS-DMA (buffer_load ... lds, which needs SGPR operands) was
  wrapped in a readfirstlane waterfall loop and the kernel ran at half speed;
* scratch spills in the tile loop count in vmcnt, so the kernel's hand-counted
  `s_waitcnt vmcnt(N)` drains the DMA prefetch (44 vmcnt(0) instead of ~20).
Two instruction-count guards on the hash loop itself:
* the xor3 written as inline asm made the hazard recognizer pad it with s_nop
  (76 per 128 bytes); the builtin does not;
* in the rotated buzhash frame (TOP) the candidate test is a bare v_min3, no v_and.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "kopia_amd", "csrc", "kcdc_kernels.hip")
HIPCC = "/opt/rocm/bin/hipcc"
KERNELS = ["_ZN4kcdc3dev23split_batch_pipe_kernelILb1EEEvNS0_9BatchArgsE",  # <TOP = true>
           "_ZN4kcdc3dev20cand_scan_dma_kernelILb1EEEvNS0_9BatchArgsENS0_8LongArgsE"]  # long-path scan


def _blocks(asm: str, kernel: str):
    """Basic blocks of a DMA kernel: (label, [instructions])."""
    m = re.search(rf"^{kernel}:(.*?)s_endpgm", asm, re.S | re.M)
    assert m, "DMA kernel not found in the device assembly"
    out, cur = [], ["entry", []]
    out.append(cur)
    for line in m.group(1).split("\n"):
        lm = re.match(r"^(\.LBB\S+):", line)
        if lm:
            cur = [lm.group(1), []]
            out.append(cur)
        elif line.startswith("\t") and not line.strip().startswith((";", ".")):
            cur[1].append(line.strip())
    return out


@pytest.fixture(scope="module")
def dma_asm(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("asm") / "k.s"
    res = tmp_path_factory.mktemp("asm") / "res.txt"
    with open(res, "w") as rf:
        subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", SRC,
                        "-o", str(out), "-Rpass-analysis=kernel-resource-usage"], check=True, stderr=rf)
    return open(out).read(), open(res).read()


@pytest.mark.parametrize("kernel", KERNELS)
def test_dma_not_in_waterfall_loops(dma_asm, kernel):
    asm, _ = dma_asm
    for label, ins in _blocks(asm, kernel):
        if any("buffer_load_dwordx4" in i and " lds" in i for i in ins):
            assert not any(i.startswith("s_cbranch_execnz " + label) for i in ins), \
                f"LDS-DMA in a readfirstlane waterfall loop at {label}"
            assert not any(i.startswith("v_readfirstlane") for i in ins), f"readfirstlane next to LDS-DMA at {label}"


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_scratch_in_hash_or_dma_blocks(dma_asm, kernel):
    asm, _ = dma_asm
    hot = 0
    for label, ins in _blocks(asm, kernel):
        is_hash = sum(1 for i in ins if i.startswith("v_bitop3_b32")) >= 32
        is_dma = any("buffer_load_dwordx4" in i and " lds" in i for i in ins)
        hot += is_hash
        if is_hash or is_dma:
            assert not any(i.startswith("scratch_") for i in ins), f"scratch access in hot block {label}"
    assert hot >= 1, "expected the unrolled hash step"


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_vgpr_spills(dma_asm, kernel):
    _, res = dma_asm
    sect = res[res.index("Function Name: " + kernel):]
    m = re.search(r"VGPRs Spill: (\d+)", sect)
    assert m and int(m.group(1)) == 0, "VGPR spills in the DMA kernel"


@pytest.mark.parametrize("kernel", KERNELS)
def test_hash_blocks_lean(dma_asm, kernel):
    asm, _ = dma_asm
    for label, ins in _blocks(asm, kernel):
        nb = sum(1 for i in ins if i.startswith("v_bitop3_b32"))
        if nb >= 32:
            hk = [k for k, i in enumerate(ins) if i.startswith("v_bitop3_b32")]
            assert not any(i.startswith("s_waitcnt") and "vmcnt" in i for i in ins[hk[0]:hk[-1]]), \
                f"vmcnt wait among the hash instructions of {label} (drains the DMA prefetch)"
            nop = sum(1 for i in ins if i.startswith("s_nop"))
            vand = sum(1 for i in ins if i.startswith("v_and_b32"))
            assert nop <= nb // 16, f"{nop} s_nop for {nb} bytes in {label}"
            assert vand <= max(4, nb // 16), f"{vand} v_and_b32 for {nb} bytes in {label} (TOP test should be min-only)"


# ---- Rabin-Karp batch and long-path kernels (two-byte hop, round 3)
RK_KERNELS = ["_ZN4kcdc3dev21split_batch_rk_kernelENS0_9BatchArgsE",
              "_ZN4kcdc3dev19cand_scan_rk_kernelENS0_9BatchArgsENS0_8LongArgsE"]


@pytest.mark.parametrize("kernel", RK_KERNELS)
def test_rk_no_vgpr_spills(dma_asm, kernel):
    """The running candidate mins reassociated into trees (no asm barrier) and 64-bit per-lane
    coordinates live across the walk each pushed the kernel past 256 VGPRs; the spill reloads
    at every 64-byte check waited vmcnt and drained the line DMA."""
    _, res = dma_asm
    sect = res[res.index("Function Name: " + kernel):]
    m = re.search(r"VGPRs Spill: (\d+)", sect)
    assert m and int(m.group(1)) == 0, "VGPR spills in the Rabin-Karp kernel"


@pytest.mark.parametrize("kernel", RK_KERNELS)
def test_rk_hop_blocks_clean(dma_asm, kernel):
    """No scratch and no vmcnt wait among a block's table reads (the hops of the walk)."""
    asm, _ = dma_asm
    hot = 0
    for label, ins in _blocks(asm, kernel):
        rd = [k for k, i in enumerate(ins) if i.startswith("ds_read_b64")]
        if len(rd) < 16:
            continue
        hot += 1
        assert not any(i.startswith("scratch_") for i in ins[rd[0]:rd[-1]]), f"scratch among the hops of {label}"
        assert not any(i.startswith("s_waitcnt") and "vmcnt" in i for i in ins[rd[0]:rd[-1]]), \
            f"vmcnt wait among the hops of {label} (drains the line DMA)"
    assert hot >= 1, "expected the unrolled two-chain walk"


# ---- content encryption / hash / compression kernels: LDS tables are read with ds_read only
# A work-in-progress AES-GCM byte pass (round 2, before c909f3c) formed a T-table address as a
# generic pointer and faulted the GPU (hipErrorIllegalAddress in test_rfc_shaped_single[AES]).
# Every table read in these kernels must stay in the LDS address space, and none may spill.
XSRC = {"crypt": "kcdc_crypt.hip", "hash": "kcdc_hash.hip", "compress": "kcdc_compress.hip"}


@pytest.fixture(scope="module", params=sorted(XSRC))
def xasm(request, tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = os.path.join(ROOT, "kopia_amd", "csrc", XSRC[request.param])
    out = tmp_path_factory.mktemp("xasm") / "k.s"
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", src,
                    "-o", str(out)], check=True, stderr=subprocess.DEVNULL)
    return request.param, open(out).read()


def _kernel_bodies(asm: str):
    funcs = set(re.findall(r"^\s*\.type\s+(_Z[^,\s]*),@function", asm, re.M))
    for m in re.finditer(r"^(_Z[^ :]*):", asm, re.M):
        if m.group(1) not in funcs:  # a __device__ constant (e.g. the zstd FSE tables), not code
            continue
        body = re.search(rf"^{re.escape(m.group(1))}:(.*?)^\.Lfunc_end", asm, re.S | re.M)
        yield m.group(1), body.group(1)


def test_no_flat_or_scratch_access(xasm):
    what, asm = xasm
    n = 0
    for name, body in _kernel_bodies(asm):
        n += 1
        flat = re.findall(r"^\s*(flat_\w+)", body, re.M)
        assert not flat, f"{name}: generic (flat) memory access {flat[:3]}"
        assert not re.search(r"^\s*scratch_", body, re.M), f"{name}: scratch access (spill or stack array)"
    assert n >= 1, f"no kernels found in {what}"


def test_gcm_tables_read_from_lds(xasm):
    what, asm = xasm
    if what != "crypt":
        pytest.skip("AES-GCM kernels live in kcdc_crypt.hip")
    seen = 0
    for name, body in _kernel_bodies(asm):
        if "gcm_units_kernel" in name or "gcm_prep_kernel" in name:
            seen += 1
            assert len(re.findall(r"^\s*ds_read", body, re.M)) >= 256, f"{name}: table lookups not in LDS"
    assert seen == 4


# ---- the ticket a wave holds while it helps
# Round 4's Rabin-Karp port lost streams because the backend (AMD clang 22.0.0git roc-7.2.0) placed
# the loop-carried `take_t = cur.cap` copy on only one of the help task's two ending paths: a task
# that ended because its owner closed the region re-entered the blocking take with the previous
# take_t (~0, "take a fresh ticket") and its held ticket was never presented again.  Both batch
# kernels now take the ticket back from memory (held_get) in the help task's end block; the load's
# value is defined after the paths join, so no per-path copy can carry a stale one.
HELD_KERNELS = ["_ZN4kcdc3dev23split_batch_pipe_kernelILb1EEEvNS0_9BatchArgsE",
                "_ZN4kcdc3dev23split_batch_pipe_kernelILb0EEEvNS0_9BatchArgsE",
                "_ZN4kcdc3dev21split_batch_rk_kernelENS0_9BatchArgsE"]


@pytest.mark.parametrize("kernel", HELD_KERNELS)
def test_help_end_reads_held_ticket_from_memory(dma_asm, kernel):
    asm, _ = dma_asm
    sites = []
    for label, ins in _blocks(asm, kernel):
        for k, i in enumerate(ins):
            if i.startswith("global_load_dwordx2") and i.endswith("offset:16 sc1"):
                dst = i.split()[1].rstrip(",")
                lo = dst[2:-1].split(":")[0] if dst.startswith("v[") else dst[1:]
                sites.append((label, any(j.startswith("v_readlane_b32") and f", v{lo}, 0" in j for j in ins[k:])))
    assert len(sites) == 1, f"expected one held-ticket load in {kernel}, found {sites}"
    assert sites[0][1], f"the held-ticket load's value is not read back in its own block ({sites[0][0]})"
