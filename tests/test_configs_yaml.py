"""configs.dm_config(name) against the reference's own config/DM/<name>.yaml
(yaml.safe_load): every key FlowDiffusion / GaussianDiffusion / the eval driver
read must match. Skipped where /root/reference is absent (the GPU box)."""
import importlib
import os

import pytest

from tests.golden_inputs import PKG

yaml = pytest.importorskip('yaml')
configs = importlib.import_module(PKG + ".configs")
pkg = importlib.import_module(PKG)
REF = '/root/reference/config/DM'

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason='reference configs absent')


@pytest.mark.parametrize('name', ['bair', 'kth', 'cityscapes', 'smmnist', 'ucf'])
def test_dm_config_matches_reference_yaml(name):
    with open(os.path.join(REF, f'{name}.yaml')) as f:
        ref = yaml.safe_load(f)
    mine = configs.dm_config(name)
    assert mine['flow_params']['model_params'] == ref['flow_params']['model_params']
    for k, v in mine['diffusion_params']['model_params'].items():
        assert ref['diffusion_params']['model_params'][k] == v, k
    assert set(ref['diffusion_params']['model_params']) == set(mine['diffusion_params']['model_params'])
    ds, rds = mine['dataset_params'], ref['dataset_params']
    assert ds['frame_shape'] == rds['frame_shape']
    for part in ('train_params', 'valid_params'):
        for k in ('type', 'cond_frames', 'pred_frames'):
            assert ds[part][k] == rds[part][k], (part, k)


@pytest.mark.parametrize('name', ['bair', 'cityscapes'])
def test_load_dm_config_reads_reference_yaml(name):
    """load_dm_config(path) is the drop-in for valid.py's yaml load + the CLI override."""
    path = os.path.join(REF, f'{name}.yaml')
    cfg = configs.load_dm_config(path, estimate_occlusion_map=False)
    assert cfg['flow_params']['model_params']['generator_params']['pixelwise_flow_predictor_params'][
        'estimate_occlusion_map'] is False
    assert cfg['dataset_params']['frame_shape'] == configs.dm_config(name)['dataset_params']['frame_shape']


def test_flow_diffusion_by_module_fixes_the_wrapper():
    """valid.py picks the sampling wrapper by importing FlowDiffusion from the module
    named by DM_arch; FLOW_DIFFUSION_BY_MODULE is the same switch as a class lookup."""
    cfg = pkg.configs.dm_config('bair')
    want = {'VideoFlowDiffusion_multi_w_ref': 'multi_w_ref',
            'VideoFlowDiffusion_multi_w_ref_u22': 'multi_w_ref_u22',
            'VideoFlowDiffusion_multi1248': 'multi1248'}
    assert set(pkg.FLOW_DIFFUSION_BY_MODULE) == set(want)
    for mod, cls in pkg.FLOW_DIFFUSION_BY_MODULE.items():
        fd = cls(config=cfg, is_train=False)
        assert isinstance(fd, pkg.FlowDiffusion) and fd.wrapper == want[mod]
    with pytest.raises(ValueError):
        pkg.FlowDiffusionMultiWRef(config=cfg, is_train=False, wrapper='multi1248')
