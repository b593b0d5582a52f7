"""The config/DM/<dataset>.yaml surface FlowDiffusion reads, restated per
dataset (values from the reference's config/DM/{bair,kth,cityscapes,smmnist,ucf}.yaml),
plus the wrapper / denoiser pairing the eval scripts use.

`dm_config(name)` returns a nested dict with the same keys as the YAML
(dataset_params, flow_params.model_params, diffusion_params.model_params), so
`FlowDiffusion(config=dm_config('bair'), ...)` and a `yaml.safe_load`ed file
are interchangeable.
"""
import copy

_COMMON_FLOW = {
    'num_channels': 3, 'estimate_affine': True, 'revert_axis_swap': True,
    'bg_predictor_params': {'block_expansion': 32, 'max_features': 1024, 'num_blocks': 5, 'bg_type': 'affine'},
    'region_predictor_params': {'temperature': 0.1, 'block_expansion': 32, 'max_features': 1024,
                                'scale_factor': 0.5, 'num_blocks': 5, 'pca_based': True, 'pad': 0,
                                'fast_svd': False},
    'generator_params': {'block_expansion': 64, 'max_features': 512, 'num_down_blocks': 2,
                         'num_bottleneck_blocks': 6, 'skips': True,
                         'pixelwise_flow_predictor_params': {'block_expansion': 64, 'max_features': 1024,
                                                             'num_blocks': 5, 'scale_factor': 0.5,
                                                             'use_deformed_source': True,
                                                             'use_covar_heatmap': True,
                                                             'estimate_occlusion_map': True}},
}

# name: (frame_shape, train (cond, pred), valid (cond, pred), num_regions, scale_factor, bg_type,
#        (FlowDiffusion wrapper module, Unet3D module))
_DATASETS = {
    'bair': (64, (2, 10), (2, 28), 10, 0.5, 'affine',
             ('VideoFlowDiffusion_multi_w_ref', 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_u12')),
    'kth': (64, (10, 20), (10, 40), 10, 0.5, 'affine',
            ('VideoFlowDiffusion_multi_w_ref', 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada')),
    'cityscapes': (128, (2, 5), (2, 28), 20, 0.25, 'perspective',
                   ('VideoFlowDiffusion_multi_w_ref_u22', 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada_u22')),
    'smmnist': (64, (10, 5), (10, 10), 10, 0.5, 'affine',
                ('VideoFlowDiffusion_multi1248', 'DenoiseNet_STWAtt_w_wo_ref_adaptor_cross_multi')),
    'ucf': (64, (4, 8), (4, 16), 64, 0.5, 'affine',
            ('VideoFlowDiffusion_multi_w_ref_u22', 'DenoiseNet_STWAtt_w_w_ref_adaptor_cross_multi_traj_ada_u22')),
}

# valid_params.type (kth.yaml names its split 'valid')
_VALID_TYPE = {'kth': 'valid'}

WRAPPERS = {'VideoFlowDiffusion_multi_w_ref': 'multi_w_ref', 'VideoFlowDiffusion_multi_w_ref_u22': 'multi_w_ref_u22',
            'VideoFlowDiffusion_multi1248': 'multi1248'}


def dm_config(name, pred_frames=None, sampling_timesteps=10, estimate_occlusion_map=True):
    """The YAML-equivalent config dict for `name`. `pred_frames` overrides the
    per-round tp (train_params.pred_frames, e.g. 14 for the BAIR 2 x 14 -> 28
    benchmark); `estimate_occlusion_map` plays the eval CLI flag (valid.py:81)."""
    S, (tc, tp), (vc, vp), R, scale, bg, _ = _DATASETS[name]
    fp = copy.deepcopy(_COMMON_FLOW)
    fp['num_regions'] = R
    fp['bg_predictor_params']['bg_type'] = bg
    fp['region_predictor_params']['scale_factor'] = scale
    pf = fp['generator_params']['pixelwise_flow_predictor_params']
    pf['scale_factor'] = scale
    pf['estimate_occlusion_map'] = bool(estimate_occlusion_map)
    return {
        'experiment_name': f'{name}{S}',
        'dataset_params': {'frame_shape': S,
                           'train_params': {'type': 'train', 'cond_frames': tc,
                                            'pred_frames': tp if pred_frames is None else pred_frames},
                           'valid_params': {'type': _VALID_TYPE.get(name, 'test'), 'cond_frames': vc,
                                            'pred_frames': vp}},
        'flow_params': {'model_params': fp},
        'diffusion_params': {'model_params': {'null_cond_prob': 0.0, 'use_residual_flow': False,
                                              'only_use_flow': False, 'sampling_timesteps': sampling_timesteps,
                                              'loss_type': 'l2', 'ada_layers': 'auto'}},
    }


def load_dm_config(path, estimate_occlusion_map=None):
    """A config/DM YAML file as valid.py loads it (yaml.safe_load), with the
    `--estimate_occlusion_map` CLI override applied (valid.py:78-81) when given."""
    import yaml
    with open(path) as f:
        cfg = yaml.safe_load(f)
    if estimate_occlusion_map is not None:
        pf = cfg['flow_params']['model_params']['generator_params']['pixelwise_flow_predictor_params']
        pf['estimate_occlusion_map'] = bool(estimate_occlusion_map)
    return cfg


def dm_arch(name):
    """(FlowDiffusion wrapper key for lfae.FlowDiffusion, Unet3D module name) used for `name`."""
    wrapper, unet = _DATASETS[name][6]
    return WRAPPERS[wrapper], unet
