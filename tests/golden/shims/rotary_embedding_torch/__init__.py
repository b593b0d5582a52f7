"""Restatement of rotary-embedding-torch 0.8.3 (pinned in the reference's
environment.yml; absent offline) -- only what the reference calls:
`RotaryEmbedding(dim)` with the `freqs` parameter (so state_dict keys match)
and `rotate_queries_or_keys(t)` along the second-to-last (sequence) axis.

Published algorithm (lang mode, theta = 1e4):
  freqs[i]  = 1 / theta ** (2i / dim),  i < dim/2          (fp32)
  angle[n]  = n * freqs, repeated interleaved (f0 f0 f1 f1 ...)
  out       = t * cos(angle) + rotate_half(t) * sin(angle)
  rotate_half pairs (x1, x2) -> (-x2, x1) on interleaved pairs.
Parity at this boundary is unpinned (no reference test fixes it).
Test harness only."""
import torch
from torch import nn
from einops import rearrange, repeat


def rotate_half(x):
    x = rearrange(x, '... (d r) -> ... d r', r=2)
    x1, x2 = x.unbind(dim=-1)
    x = torch.stack((-x2, x1), dim=-1)
    return rearrange(x, '... d r -> ... (d r)')


def apply_rotary_emb(freqs, t, start_index=0, scale=1.):
    rot_dim = freqs.shape[-1]
    end_index = start_index + rot_dim
    t_left, t_mid, t_right = t[..., :start_index], t[..., start_index:end_index], t[..., end_index:]
    t_mid = (t_mid * freqs.cos() * scale) + (rotate_half(t_mid) * freqs.sin() * scale)
    return torch.cat((t_left, t_mid, t_right), dim=-1)


class RotaryEmbedding(nn.Module):
    def __init__(self, dim, theta=10000, learned_freq=False):
        super().__init__()
        freqs = 1. / (theta ** (torch.arange(0, dim, 2)[:(dim // 2)].float() / dim))
        self.freqs = nn.Parameter(freqs, requires_grad=learned_freq)

    def rotate_queries_or_keys(self, t, seq_dim=-2):
        seq_len = t.shape[seq_dim]
        pos = torch.arange(seq_len, device=t.device, dtype=t.dtype)
        freqs = torch.einsum('..., f -> ... f', pos.type(self.freqs.dtype), self.freqs)
        freqs = repeat(freqs, '... n -> ... (n r)', r=2)
        return apply_rotary_emb(freqs, t)
