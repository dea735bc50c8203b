"""Plain-PyTorch reference math for every fused op.

These functions reproduce the reference model's numerics (reference model.py) and are used
(1) as the fp32 oracle in the kernel tests and (2) as the implementation on CPU tensors (the
CPU/gloo configuration of BASELINE.json). They are never used for GPU tensors.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def precompute_freqs_cis(dim: int, end: int, theta: float = 10000.0) -> torch.Tensor:
    """complex64 [end, dim/2] rotation table, identical to reference model.py:52-72."""
    freqs = 1.0 / (theta ** (torch.arange(0, dim, 2)[: (dim // 2)].float() / dim))
    t = torch.arange(end, device=freqs.device)
    freqs = torch.outer(t, freqs).float()
    return torch.polar(torch.ones_like(freqs), freqs)


def rope_table(freqs_cis: torch.Tensor) -> torch.Tensor:
    """fp32 [S, D/2, 2] = (cos, sin), the layout the HIP RoPE kernel reads."""
    return torch.view_as_real(freqs_cis).contiguous()


def up(x: torch.Tensor) -> torch.Tensor:
    """Opmath of ``x``: fp32 for 16-bit/fp32 tensors, fp64 for fp64 (fp64 models stay fp64)."""
    return x.to(torch.promote_types(x.dtype, torch.float32))


# ---------------------------------------------------------------------------------------
def rmsnorm_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    """reference model.py:44-49"""
    xf = up(x)
    out = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).type_as(x)
    return out * w


def rmsnorm_fwd(x, delta, w, eps):
    """(h, y, rstd) with h = round(x + delta) when delta is given."""
    h = x if delta is None else (x + delta)
    hf = up(h)
    rstd = torch.rsqrt(hf.pow(2).mean(-1) + eps)
    y = (hf * rstd.unsqueeze(-1)).to(h.dtype) * w
    return h, y, rstd.reshape(-1)


def rmsnorm_bwd(dy, h, w, rstd, dres):
    """returns (dx, dw_fp32) with the same rounding points as the HIP kernel."""
    D = h.shape[-1]
    hf = up(h).reshape(-1, D)
    dyf = up(dy).reshape(-1, D)
    r = rstd.reshape(-1, 1)
    nb = up((hf * r).to(h.dtype))
    dw = (dyf * nb).sum(0)
    g = up((dyf * up(w)).to(h.dtype))
    dot = (g * hf).sum(-1, keepdim=True)
    dx = (r * (g - hf * (r * r * dot / D))).to(h.dtype)
    if dres is not None:
        dx = dx + dres.reshape(-1, D)
    return dx.reshape(h.shape), dw


def rope_inplace_2d(x2d: torch.Tensor, ncols: int, tab: torch.Tensor, head_dim: int, seq_len: int,
                    inverse: bool = False):
    """Rotate the first `ncols` columns of every row (heads of size head_dim), interleaved pairs."""
    T = x2d.shape[0]
    v = up(x2d[:, :ncols]).reshape(T // seq_len, seq_len, ncols // head_dim, head_dim // 2, 2)
    c = tab[:seq_len, :, 0].view(1, seq_len, 1, head_dim // 2)
    s = tab[:seq_len, :, 1].view(1, seq_len, 1, head_dim // 2)
    if inverse:
        s = -s
    a, b = v[..., 0], v[..., 1]
    out = torch.stack([a * c - b * s, a * s + b * c], dim=-1)
    x2d[:, :ncols] = out.reshape(T, ncols).to(x2d.dtype)


def apply_rotary_emb_ref(xq, xk, freqs_cis):
    """reference model.py:101-127 ([B, S, H, D] tensors)"""
    xq_ = torch.view_as_complex(up(xq).reshape(*xq.shape[:-1], -1, 2))
    xk_ = torch.view_as_complex(up(xk).reshape(*xk.shape[:-1], -1, 2))
    fc = freqs_cis[: xq.shape[1]].view(1, xq.shape[1], 1, xq_.shape[-1])
    xq_out = torch.view_as_real(xq_ * fc).flatten(3)
    xk_out = torch.view_as_real(xk_ * fc).flatten(3)
    return xq_out.type_as(xq), xk_out.type_as(xk)


def attention_ref(q, k, v, causal: bool = True, scale: Optional[float] = None):
    """[B, S, H, D] in/out; GQA by repeating kv heads (reference model.py:130-139, 217-229)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    if Hkv != Hq:
        k = k.repeat_interleave(Hq // Hkv, dim=2)
        v = v.repeat_interleave(Hq // Hkv, dim=2)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                       is_causal=causal, scale=scale)
    return o.transpose(1, 2).contiguous()


def attention_lse_ref(q, k, v, causal=True, scale=None):
    """fp32 attention output + natural-log LSE [B, H, S] (oracle for the HIP kernel)."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    kk = up(k).repeat_interleave(Hq // Hkv, dim=2)
    vv = up(v).repeat_interleave(Hq // Hkv, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", up(q), kk) * scale
    if causal:
        m = torch.ones(S, S, dtype=torch.bool, device=q.device).triu(1)
        s = s.masked_fill(m, float("-inf"))
    lse = torch.logsumexp(s, dim=-1)
    p = torch.softmax(s, dim=-1)
    o = torch.einsum("bhqk,bkhd->bqhd", p, vv)
    return o, lse


def swiglu_ref(g, u):
    """reference model.py:269: silu(w1 x) * w3 x"""
    return F.silu(g) * u


def swiglu_bwd_ref(dy, g, u):
    gf, uf, dyf = up(g), up(u), up(dy)
    sg = torch.sigmoid(gf)
    a = up((gf * sg).to(g.dtype))
    da = up((dyf * uf).to(g.dtype))
    du = dyf * a
    dg = da * sg * (1 + gf * (1 - sg))
    return dg.to(g.dtype), du.to(g.dtype)


def cross_entropy_ref(logits, labels, ignore_index: int = -100):
    """reference train.py:253,263-266: sum-reduced CE on fp32 logits / #non-ignored labels."""
    n = labels.ne(ignore_index).sum()
    loss = F.cross_entropy(up(logits.flatten(0, -2)), labels.flatten(), reduction="sum",
                           ignore_index=ignore_index)
    return loss / n
