"""bench.py prices each roofline kernel against the dense MFMA peak of the arithmetic it runs,
read from its template arguments (round-4 VERDICT: attn_core_kernel was priced as fp32 by a
name prefix, although X3 = true is f16x3 and X3 = false is bf16)."""
import pytest

import bench

F16X3 = 2516.6 / 3


@pytest.mark.parametrize('kname,precision,arith,peak', [
    ('attn_core_kernel<0, true, 2>', 'f16x3', 'f16x3', F16X3),
    ('attn_core_kernel<1, true, 1>', 'bf16_attn', 'f16x3', F16X3),
    ('attn_core_kernel<0, false, 2>', 'bf16_attn', 'bf16', 2516.6),
    ('attn_core_kernel<1, false, 1>', 'f16x3', 'bf16', 2516.6),
    ('stw64_x3_kernel<64, 16, 8, false>', 'f16x3', 'f16x3', F16X3),
    ('attn_x3_kernel<64, 0, 32, 8, true, false>', 'f16x3', 'f16x3', F16X3),
    ('attn_fused_kernel<64, 0, 2, 16>', 'f16x3', 'fp32', 157.3),
    ('window_attn_kernel', 'f16x3', 'fp32', 157.3),
    ('conv_x3_kernel<3, 1, 64, 256, 1, 4, 4, 2, true, 2, false, false, 0, false, false>', 'fp32', 'f16x3', F16X3),
    ('cross_attn_x3p_kernel<1>', 'f16x3', 'f16x3', F16X3),
    ('xpath_x3_kernel<2, 2>', 'f16x3', 'f16x3', F16X3),
    ('conv_kernel<3, 64>', 'f16x3', 'fp32', 157.3),
])
def test_peak_by_template(kname, precision, arith, peak):
    assert bench.kernel_arith(kname, precision) == arith
    assert bench.kernel_peak(arith) == pytest.approx(peak)


@pytest.mark.parametrize('kname', ['stw64_x3_kernel<64, 32, 8, true>', 'attn_x3_kernel<64, 1, 32, 8, true, true>'])
def test_mixed_bf16_attention_peak(kname):
    """The fused kernels in BF16_ATTN: qkv / proj on f16x3, QK^T / PV on bf16 -> the FLOP-weighted
    harmonic peak, between the two and equal to either at the ends."""
    assert bench.kernel_arith(kname, 'bf16_attn') == 'f16x3+bf16'
    assert bench.kernel_peak('f16x3+bf16', 0.0) == pytest.approx(F16X3)
    assert bench.kernel_peak('f16x3+bf16', 1.0) == pytest.approx(2516.6)
    f = 4 * 64 / (8 * 64 + 4 * 64)  # level-0 64-token windows, C 64
    p = bench.kernel_peak('f16x3+bf16', f)
    assert F16X3 < p < 2516.6
    assert 1 / p == pytest.approx((1 - f) / F16X3 + f / 2516.6)


@pytest.mark.parametrize('kname,arith', [
    ('stw64_x3_kernel<64, 32, 8, true, true>', 'f16x3+bf16'),
    ('stw64_x3_kernel<128, 16, 4, false, false>', 'f16x3'),
    ('attn_core_kernel<0, true, 2, 16>', 'f16x3'),
    ('attn_core_kernel<0, false, 1, 32>', 'bf16'),
])
def test_current_template_arity(kname, arith):
    """The names the library reports today (five stw64 / four attn_core template arguments)."""
    assert bench.kernel_arith(kname, 'fp32') == arith


def test_note_kernel_formats_are_parsed_by_template():
    """Every note_kernel format string in csrc/ for the families kernel_arith reads by argument
    (attn_core, attn_x3, stw64) parses by its template, not the by-name fallback: a format with a
    new argument count must fail here rather than price a bf16 kernel as f16x3."""
    import glob
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = glob.glob(os.path.join(root, '*_amd', 'csrc', '*.hip'))
    assert csrc
    seen = set()
    for path in csrc:
        for m in re.finditer(r'note_kernel\("((\w+)<[^"]*>)"', open(path).read()):
            fmt, ident = m.group(1), m.group(2)
            if ident not in ('attn_core_kernel', 'attn_x3_kernel', 'stw64_x3_kernel'):
                continue
            seen.add(ident)
            name = fmt.replace('%d', '64').replace('%s', 'true')
            # by template: the bf16 flag set -> never the precision fallback ('fp32' here)
            assert bench.kernel_arith(name, 'fp32') in ('bf16', 'f16x3+bf16', 'f16x3'), fmt
            assert bench.kernel_arith(name, 'fp32') != 'f16x3' or ident == 'attn_core_kernel', fmt
    assert seen == {'attn_core_kernel', 'attn_x3_kernel', 'stw64_x3_kernel'}
