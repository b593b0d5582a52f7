"""Stand-in for timm 0.4.5 (absent offline). The reference uses `trunc_normal_`
at init only and never instantiates DropPath on the sampling path."""
import torch
from torch import nn


def trunc_normal_(tensor, mean=0., std=1., a=-2., b=2.):
    with torch.no_grad():
        return nn.init.trunc_normal_(tensor, mean=mean, std=std, a=a, b=b)


class DropPath(nn.Identity):
    def __init__(self, *args, **kwargs):
        super().__init__()
