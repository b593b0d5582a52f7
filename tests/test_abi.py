"""The C-ABI library loads (no GPU needed) and exports every symbol that
include/extdm.h declares; the package refuses CPU tensors (no fallback)."""
import ctypes
import importlib
import os
import re

import pytest
import torch

from tests.golden_inputs import PKG

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pkg = importlib.import_module(PKG)


def declared():
    src = open(os.path.join(REPO, 'include', 'extdm.h')).read()
    return sorted(set(re.findall(r'\b(extdm_[a-z_]+)\s*\(', src)))


def test_header_matches_binding_list():
    assert declared() == sorted(pkg._lib.EXPORTS)


def test_library_exports_all_symbols():
    if not os.path.exists(pkg._lib.LIB_PATH):
        pytest.skip('library not built here (run __graft_entry__.build())')
    lib = ctypes.CDLL(pkg._lib.LIB_PATH)
    for name in declared():
        assert hasattr(lib, name), name


def test_cpu_tensors_are_rejected():
    u = pkg.Unet3D(dim=16, channels=512, dim_mults=(1, 2, 4, 4), cond_num=2, pred_num=6, framesize=16)
    x = torch.zeros(1, 3, 6, 16, 16)
    with pytest.raises(RuntimeError, match='ROCm device'):
        u(x, torch.zeros(1, dtype=torch.long), torch.zeros(1, 3, 2, 16, 16), cond_fea=torch.zeros(1, 256, 8, 8, 8))
