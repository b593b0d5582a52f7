"""The package's state_dict layout equals the reference's (key order, shapes)."""
import importlib
import json
import os

import pytest

from tests.golden_inputs import CONFIGS, GEN_CFG, PKG

spec = importlib.import_module(PKG + '.spec')
GOLD = os.path.join(os.path.dirname(__file__), 'golden')


@pytest.mark.parametrize('name', list(CONFIGS))
def test_unet_keys(name):
    ref = json.load(open(os.path.join(GOLD, 'unet_keys.json')))[name]
    mine = [[n, list(s), d] for n, s, d in spec.unet_spec(CONFIGS[name])]
    assert mine == ref


def test_generator_keys():
    ref = json.load(open(os.path.join(GOLD, 'generator_keys.json')))
    mine = [[n, list(s)] for n, s, d in spec.generator_spec(GEN_CFG)]
    assert mine == ref
