"""Stand-in for einops_exts 0.0.4 (absent offline): only `rearrange_many`,
the one name the reference imports (DenoiseNet_*.py:10). Test harness only."""
from einops import rearrange


def rearrange_many(tensors, pattern, **kwargs):
    return [rearrange(t, pattern, **kwargs) for t in tensors]
