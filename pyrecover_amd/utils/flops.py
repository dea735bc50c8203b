"""Parameter / FLOP accounting (reference utils.py:30-56).

``num_flop_per_token`` keeps the reference formula ``6*N + 12*L*H*head_dim*S`` (N = non-embedding
params). Unlike the reference (defect D9: under DDP its ``children()`` scan misses the embedding),
callers pass the unwrapped model's count, so the value is the same for any world size.
"""
from __future__ import annotations

import torch

MI355X_PEAK_BF16_DENSE = 2.5e15  # FLOP/s, dense (no sparsity)
H100_PEAK_BF16_DENSE = 989e12    # the reference's MFU denominator (train.py:287)


def get_num_params(model: torch.nn.Module, exclude_embedding: bool = False) -> int:
    m = getattr(model, "module", model)
    n = sum(p.numel() for p in m.parameters())
    if exclude_embedding:
        n -= sum(p.numel() for mod in m.modules() if isinstance(mod, torch.nn.Embedding) for p in mod.parameters())
    return n


def num_flop_per_token(num_params: int, cfg) -> int:
    l, h, q, t = cfg.n_layers, cfg.n_heads, cfg.dim // cfg.n_heads, cfg.seq_len
    return 6 * num_params + 12 * l * h * q * t


get_num_flop_per_token = num_flop_per_token
