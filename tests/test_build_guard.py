"""The device-code guard of mapache_amd/build.py.

* VGPR exact fills: a kernel whose registers fill its 8-register allocation
  exactly is rejected unless documented (the headline scan; rocPRIM library
  kernels, none of which the product launches);
* the static waitcnt audit (mapache_amd/devaudit.py): a register named while a
  load into it may still be outstanding is flagged, in-order write-after-write
  is not, LDS/SMEM counter semantics and loops are modelled;
* the kernel descriptor decoded from a real code object agrees with the
  assembly's next_free_vgpr;
* the shipped library passed the guard.
"""
import os
import subprocess

import pytest

from mapache_amd import build as B
from mapache_amd import devaudit as D


def _asm(tmp_path, kernels):
    body = []
    for name, v in kernels:
        body.append(f"\t.amdhsa_kernel {name}\n\t\t.amdhsa_next_free_vgpr {v}\n\t\t.amdhsa_accum_offset {v}\n"
                    f"\t.end_amdhsa_kernel\n")
    p = tmp_path / "x-hip-amdgcn-amd-amdhsa-gfx950.s"
    p.write_text("".join(body))
    (tmp_path / "x-host-x86_64-unknown-linux-gnu.s").write_text("\t.amdhsa_kernel _ZN4mcdc9k_ignoredEv\n"
                                                                 "\t\t.amdhsa_next_free_vgpr 8\n\t.end_amdhsa_kernel\n")
    return str(tmp_path)


def test_exact_fills_flagged(tmp_path):
    d = _asm(tmp_path, [("_ZN4mcdc6k_emitILi16EEEvNS_4WorkENS_9DevParamsEjj", 184),
                        ("_ZN4mcdc6k_emitILi16EEEvNS_4WorkENS_9DevParamsEjjX", 185),
                        ("_ZN4mcdc8k_scan_qILi4096ELi2ELb1EEEvNS_4WorkE", 128),
                        ("_ZN4mcdc8k_scan_qILi4096ELi2ELb0EEEvNS_4WorkE", 112),
                        ("_ZN7rocprim6kernelEv", 64)])
    rep = B.vgpr_report(d)
    assert len(rep) == 4  # only mcdc kernels, only device assembly
    bad = B.exact_fills(rep)
    # no exemptions since round 4: the headline scan at 128 is flagged too
    assert [k for k, _ in bad] == ["_ZN4mcdc6k_emitILi16EEEvNS_4WorkENS_9DevParamsEjj",
                                   "_ZN4mcdc8k_scan_qILi4096ELi2ELb1EEEvNS_4WorkE",
                                   "_ZN4mcdc8k_scan_qILi4096ELi2ELb0EEEvNS_4WorkE"]


def _unit(body):
    ins, lab = D.parse(body.strip("\n").split("\n"))
    return [h for h in D.analyse(ins, lab, "u")]


def test_waitcnt_raw_flagged_and_covered():
    h = _unit("""
    global_load_dwordx2 v[2:3], v[0:1], off
    v_add_u32_e32 v4, v2, v5
""")
    assert len(h) == 1 and h[0][3] == [2] and h[0][5] == "raw"
    assert not _unit("""
    global_load_dwordx2 v[2:3], v[0:1], off
    global_load_dword v6, v[0:1], off offset:8
    s_waitcnt vmcnt(1)
    v_add_u32_e32 v4, v2, v3
""")
    # vmcnt(1) leaves the newer load outstanding
    h = _unit("""
    global_load_dword v2, v[0:1], off
    global_load_dword v6, v[0:1], off offset:8
    s_waitcnt vmcnt(1)
    v_add_u32_e32 v4, v6, v2
""")
    assert [x[3] for x in h] == [[6]]


def test_waitcnt_lds_smem_and_waw():
    # LDS returns in order: lgkmcnt(1) completes all but the newest LDS read,
    # even with a scalar load outstanding (it can only be among the 1)
    assert not _unit("""
    s_load_dword s4, s[0:1], 0x0
    ds_read_b32 v1, v0
    ds_read_b32 v2, v0 offset:4
    s_waitcnt lgkmcnt(1)
    v_mov_b32_e32 v3, v1
""")
    h = _unit("""
    ds_read_b32 v1, v0
    ds_read_b32 v2, v0 offset:4
    s_waitcnt lgkmcnt(1)
    v_mov_b32_e32 v3, v2
""")
    assert [x[3] for x in h] == [[2]]
    # a second load into the same register of the same in-order queue: benign
    h = _unit("""
    global_load_dword v1, v[8:9], off
    global_load_dword v1, v[8:9], off offset:4
    s_waitcnt vmcnt(0)
    v_mov_b32_e32 v3, v1
""")
    assert [x[5] for x in h] == ["waw-in-order"]


def test_waitcnt_across_loop_back_edge():
    # the load at the loop bottom is consumed at the loop top of the next trip
    h = _unit("""
    s_mov_b32 s2, 4
.LBB0_1:
    v_add_u32_e32 v4, v2, v4
    global_load_dword v2, v[0:1], off
    s_add_i32 s2, s2, -1
    s_cmp_lg_u32 s2, 0
    s_cbranch_scc1 .LBB0_1
    s_endpgm
""")
    assert [(x[3], x[5]) for x in h] == [([2], "raw"), ([2], "waw-in-order")]
    assert not _unit("""
    s_mov_b32 s2, 4
.LBB0_1:
    s_waitcnt vmcnt(0)
    v_add_u32_e32 v4, v2, v4
    global_load_dword v2, v[0:1], off
    s_add_i32 s2, s2, -1
    s_cmp_lg_u32 s2, 0
    s_cbranch_scc1 .LBB0_1
    s_endpgm
""")


KSRC = r"""
#include <hip/hip_runtime.h>
#include <stdint.h>
namespace mcdc {
__global__ void k_plain(const uint64_t *a, uint64_t *b) {
  b[threadIdx.x] = a[threadIdx.x] * 3 + 1;
}
__global__ void k_padded(const uint64_t *a, uint64_t *b) {
  asm volatile("v_mov_b32 v15, 0" ::: "v15");
  b[threadIdx.x] = a[threadIdx.x] ^ 5;
}
}
"""


def test_descriptor_decoded_from_code_object(tmp_path):
    """A real gfx950 code object: the descriptor's granulated VGPR count equals
    next_free_vgpr rounded to 8, and a kernel that names v15 is an exact fill
    (16 of 16) that device_guard rejects by name."""
    src = tmp_path / "k.hip"
    src.write_text(KSRC)
    r = subprocess.run([B.HIPCC, "-O3", f"--offload-arch={B.ARCH}", "-save-temps", "-c", "-o", "k.o", "k.hip"],
                       cwd=tmp_path, capture_output=True, text=True)
    if r.returncode:
        pytest.skip("hipcc unavailable: " + r.stderr[-300:])
    rows, hz = D.audit(str(tmp_path), quiet=True)
    ks = {r["name"]: r for r in rows if r["kernel"]}
    assert len(ks) == 2
    for r in ks.values():
        assert r["alloc"] == (r["next_free_vgpr"] + 7) // 8 * 8
    pad = [r for n, r in ks.items() if "k_padded" in n][0]
    assert pad["next_free_vgpr"] == 16 and pad["alloc"] == 16 and pad["top"] == 15
    problems, _ = B.device_guard(str(tmp_path))
    assert any("k_padded" in p and "exactly" in p for p in problems)
    assert not any("k_plain" in p for p in problems)


def test_shipped_library_was_guarded():
    """libmcdc.so is only written after the guard passed (build_lib raises
    before os.replace); the sources it was built from pad the kernels whose
    register count would otherwise fill their allocation (k_spec6 at 80), and
    no kernel of ours is exempt from the exact-fill rule (the headline scan
    was the last, round 3)."""
    src = open(os.path.join(B.HERE, "csrc", "mcdc_kernels.hip")).read()
    assert "MCDC_VGPR_PAD(80);" in src
    assert B.EXACT_FILL_OK == ()


def test_vgpr_ceiling_by_workgroup_size():
    """A descriptor may only be padded while the new allocation still lets the
    workgroup launch: 16 waves (1024 threads) share 4 SIMDs -> 128 VGPRs."""
    assert D.vgpr_ceiling(1024) == 128
    assert D.vgpr_ceiling(768) == 168
    assert D.vgpr_ceiling(512) == 256
    assert D.vgpr_ceiling(256) == 512 and D.vgpr_ceiling(64) == 512
    asm = ".max_flat_workgroup_size: 1024\n    .name:           _ZN7rocprim4kern\n"
    assert D.max_workgroup_sizes(asm) == {"_ZN7rocprim4kern": 1024}


def test_library_padding_refused_past_the_ceiling(tmp_path):
    """pad_library_fills refuses (build fails) when one more granule would make
    a library kernel's launch impossible."""
    rows = [dict(name="_ZN7rocprim4kern", kernel=True, next_free_vgpr=128, wg_size=1024)]
    with pytest.raises(RuntimeError, match="exceeds"):
        B.pad_library_fills(str(tmp_path / "none.so"), str(tmp_path), rows)


def test_descriptor_padding_in_a_linked_library(tmp_path):
    """pad_descriptors raises one kernel's allocation by a granule in a linked
    shared library (the cure of §3a, applied to rocPRIM kernels by build_lib),
    leaves the other kernel's descriptor alone, and library_allocations reads
    the result back from the library bytes."""
    src = tmp_path / "k.hip"
    src.write_text(KSRC)
    r = subprocess.run([B.HIPCC, "-O3", f"--offload-arch={B.ARCH}", "-save-temps", "-fPIC", "-c", "-o", "k.o",
                        "k.hip"], cwd=tmp_path, capture_output=True, text=True)
    if r.returncode:
        pytest.skip("hipcc unavailable: " + r.stderr[-300:])
    subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", "k.so", "k.o"], cwd=tmp_path,
                   check=True)
    lib = str(tmp_path / "k.so")
    names = {r["name"]: r for r in D.audit(str(tmp_path), quiet=True)[0] if r["kernel"]}
    pad = [n for n in names if "k_padded" in n][0]
    plain = [n for n in names if "k_plain" in n][0]
    before = D.library_allocations(lib, str(tmp_path), names)
    assert before[pad] == 16 and before[plain] == names[plain]["alloc"]
    done = D.pad_descriptors(lib, str(tmp_path), [pad])
    assert done == [(pad, 16, 24)]
    after = D.library_allocations(lib, str(tmp_path), names)
    assert after[pad] == 24 and after[plain] == before[plain]
