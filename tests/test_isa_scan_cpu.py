"""Build-time guard for the two-board heads' wrong words: the built library's
gfx950 code objects must contain no multi-dword LDS store whose data VGPRs were written by a
packed-FP32 VALU instruction (v_pk_add / v_pk_mul / v_pk_fma _f32) in the 3 instructions before
it (scripts/ds_war_scan.py rule 2).  Round 3's heads (the val_fc1 partial-sum quad paired by
the compiler into v_pk_*_f32 chains) have that pattern at each of their 30 partial-sum
stores, and stored wrong words in lanes 48-63 with two workgroups per CU
(profiles/r04_heads_war.json, profiles/r05_heads_paired_tests.txt); the shipped heads keep the
quad's chains unpaired and the library has none.  CPU only: llvm-objdump on the .so."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import ds_war_scan as scan  # noqa: E402

LIB = os.path.join(ROOT, "alphazero-othello_amd", "libaz_othello.so")
OBJDUMP = os.path.join(scan.LLVM, "llvm-objdump")

# the round-3 heads build's partial-sum store (k_trunk_wino4<..., true>, heads_az.h paired)
BAD = """
_ZN12_GLOBAL__N_113k_trunk_wino4:
	v_pk_add_f32 v[90:91], v[90:91], v[108:109]
	v_pk_add_f32 v[92:93], v[86:87], v[88:89]
	s_add_i32 s8, 0, 0x10200
	ds_write_b128 v81, v[90:93] offset:4352
	ds_read_b128 v[86:89], v66
"""
# the shipped form: four unpaired fp32 chains, the store three VALU after the last add
GOOD = """
_ZN12_GLOBAL__N_113k_trunk_wino4:
	v_add_f32_e32 v101, v96, v101
	v_mul_u32_u24_e32 v96, 0x5f8, v153
	v_lshlrev_b32_e32 v102, 4, v166
	v_add3_u32 v96, v0, v96, v102
	ds_write_b128 v96, v[98:101] offset:4352
	ds_read_b128 v[100:103], v98
"""


def test_scanner_flags_the_failing_heads_sequence():
    bad = scan.scan_pk_stores(BAD, "snippet")
    assert [(f[2], f[3].split()[0]) for f in bad] == [(1, "v_pk_add_f32"), (2, "v_pk_add_f32")]
    assert scan.scan_pk_stores(GOOD, "snippet") == []
    # a packed result four instructions back is outside the window
    far = BAD.replace("s_add_i32 s8, 0, 0x10200",
                      "s_add_i32 s8, 0, 0x10200\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0")
    assert scan.scan_pk_stores(far, "snippet") == []


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)),
                    reason="needs the built library and llvm-objdump")
def test_library_has_no_packed_f32_result_stored_by_a_wide_lds_store():
    texts = scan.disassemble_so(LIB)
    assert texts, "no gfx950 code object found in the library"
    kernels = sum(t.count(">:\n") for _, t in texts)
    assert kernels > 50  # the whole library was disassembled
    found = []
    for name, text in texts:
        found += scan.scan_pk_stores(text, name)
    assert not found, "\n".join(f"{fn}: {prod} -> {st}" for _, fn, _, prod, st in found[:10])


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(OBJDUMP)),
                    reason="needs the built library and llvm-objdump")
def test_resident_trunk_kernels_have_no_static_lds():
    """The resident trunk's window reads use raw LDS addresses (read_rows_x in
    csrc/conv_wino4.hip): correct only while k_trunk_wino4's dynamic LDS starts at address 0,
    i.e. the kernel declares no static LDS."""
    sizes = scan.kernel_static_lds(LIB)
    trunk = {k: v for k, v in sizes.items() if "k_trunk_wino4" in k}
    assert trunk, "no k_trunk_wino4 kernel in the library's metadata"
    assert all(v == 0 for v in trunk.values()), trunk
