"""LDS layouts of the split GDN backward (csrc/gdn_fused.hip pl_sw / pl_off), checked by the bank
simulation of tools/plane_banks.py against MI355X_MICROARCH.md's LDS lane groups: the dx GEMM's
ds_read_b128 fragments and the dgamma GEMM's ds_read_b64_tr_b16 reads are conflict-free, and the
phase-A ds_write_b64 stores of gdn_bwd_x3w_kernel are at most 2-way.  CPU only."""
import importlib.util
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _mod():
    spec = importlib.util.spec_from_file_location("plane_banks", os.path.join(ROOT, "tools", "plane_banks.py"))
    m = importlib.util.module_from_spec(spec)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        spec.loader.exec_module(m)
    return m


def test_plane_swizzle_matches_the_kernel_source():
    src = open(os.path.join(ROOT, "image_compression_amd", "csrc", "gdn_fused.hip")).read()
    body = re.search(r"int pl_sw\(int m\) \{ return (.*?); \}", src).group(1)
    assert body == "(((m >> 1) & 1) << 2) | ((4 - (m >> 2)) & 3)"
    m = _mod()
    for r in range(16):
        assert m.pl_sw_new(r) == ((((r >> 1) & 1) << 2) | ((4 - (r >> 2)) & 3))


def test_plane_layout_bank_conflicts():
    m = _mod()
    res = m.simulate(m.pl_sw_new)
    assert res == (1, 1, 2), res   # b128 fragments, tr reads, phase-A stores
    assert m.simulate(m.pl_sw_old) == (1, 1, 4)
