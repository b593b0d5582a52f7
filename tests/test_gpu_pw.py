"""The register-resident-weight 1x1 kernel (pw_x3.hip: TrajWarp's linear_q / linear_o / linear_k /
linear_v, u12:806-821) against the conv_x3 1x1 launch it replaces: the BAIR u12 forward with it
(default) and with EXTDM_NO_PW=1 (consulted per launch decision, so two handles in one process)
are bit-identical (the same products in the same order); both are also checked against the
reference golden by test_gpu_parity."""
import os

import numpy as np
import pytest

from tests import parity_log
import torch

from tests.golden_inputs import CONFIGS, make_sd, unet_inputs
from tests.test_gpu_parity import gpu_eps, pkg

pytestmark = pytest.mark.gpu


def _handle(cfg, B):
    h = pkg._lib.Handle(cfg, 1000, B, 0)
    sd = make_sd(cfg)
    sd.update(pkg.schedule_buffers(1000))
    h.load_state(sd)
    h.finalize()
    return h


def test_pw_x3_matches_conv_x3():
    cfg = CONFIGS['bair']
    x, t, cond, fea = unet_inputs(cfg, B=2, seed=41)
    os.environ.pop('EXTDM_NO_PW', None)
    eps = gpu_eps(_handle(cfg, 2), x, t, cond, fea).numpy()
    os.environ['EXTDM_NO_PW'] = '1'
    try:
        ref = gpu_eps(_handle(cfg, 2), x, t, cond, fea).numpy()
    finally:
        os.environ.pop('EXTDM_NO_PW', None)
    assert np.isfinite(eps).all()
    d = np.abs(eps - ref).max()
    parity_log.check(d, 0.0, 'bitwise')
    # the contract: the same products in the same order as the conv_x3 launch -> bit-identical eps
    assert np.array_equal(eps, ref)
