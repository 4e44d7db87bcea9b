"""The VGPR exact-fill guard of mapache_amd/build.py: a kernel
whose registers fill its 8-register allocation exactly is rejected unless it is
the documented headline scan; the shipped library passes it."""
import os

from mapache_amd import build as B


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
    assert [k for k, _ in bad] == ["_ZN4mcdc6k_emitILi16EEEvNS_4WorkENS_9DevParamsEjj",
                                   "_ZN4mcdc8k_scan_qILi4096ELi2ELb0EEEvNS_4WorkE"]


def test_shipped_library_was_guarded():
    """libmcdc.so is only written after the guard passed (build_lib raises
    before os.replace); the sources it was built from pad every exact fill."""
    src = open(os.path.join(B.HERE, "csrc", "mcdc_kernels.hip")).read()
    assert "MCDC_VGPR_PAD(MCDC_EMIT_VPAD)" in src and "#define MCDC_EMIT_VPAD 184" in src
    assert "_ZN4mcdc8k_scan_qILi4096ELi2ELb1E" in B.EXACT_FILL_OK
