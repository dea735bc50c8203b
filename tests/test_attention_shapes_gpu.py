"""Attention coverage beyond the tiled bf16 fast path, against fp32 oracles:

* fp16 instantiations of every kernel (v_mfma_f32_32x32x16_f16);
* the fp32 kernels (attention_f32.hip, v_mfma_f32_32x32x2_f32) for fp32 models;
* sequence lengths that do not tile (S % 64 / S % 128 != 0): zero-padded in the binding, exact for
  causal attention and key-bounded (skv) for full attention;
* the production shapes with the DEFAULT kernel selection (no env overrides): Llama-2-7B layer
  B1 S2048 H32 D128 and Llama-3-8B layer B1 S8192 Hq32/Hkv8 D128, causal, forward + backward.
The oracle runs one kv-head group at a time in fp32 so the S=8192 score matrix stays small.
"""
import math

import pytest
import torch

from pyrecover_amd import _ext
from pyrecover_amd.ops import fused as F
from pyrecover_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _qkv(cuda, B, S, Hq, Hkv, D, dtype, seed=0):
    torch.manual_seed(seed)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=cuda).to(dtype)
    q = qkv[:, :Hq * D].view(B, S, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(B, S, Hkv, D)
    return q, k, v


def oracle(q, k, v, do, causal, scale):
    """fp32 (o, lse, dq, dk, dv), one kv head (and its query heads) at a time."""
    B, S, Hq, D = q.shape
    Hkv = k.shape[2]
    rep = Hq // Hkv
    outs = [torch.empty(B, S, Hq, D, device=q.device), torch.empty(B, Hq, S, device=q.device),
            torch.empty(B, S, Hq, D, device=q.device), torch.empty(B, S, Hkv, D, device=q.device),
            torch.empty(B, S, Hkv, D, device=q.device)]
    for h in range(Hkv):
        hs = slice(h * rep, (h + 1) * rep)
        qf = q[:, :, hs].float().requires_grad_()
        kf = k[:, :, h:h + 1].float().requires_grad_()
        vf = v[:, :, h:h + 1].float().requires_grad_()
        o, lse = R.attention_lse_ref(qf, kf, vf, causal, scale)
        o.backward(do[:, :, hs].float())
        outs[0][:, :, hs] = o.detach()
        outs[1][:, hs] = lse.detach()
        outs[2][:, :, hs] = qf.grad
        outs[3][:, :, h:h + 1] = kf.grad
        outs[4][:, :, h:h + 1] = vf.grad
        del o, lse, qf, kf, vf
    return outs


def _run(cuda, B, S, Hq, Hkv, D, causal, dtype, seed=0, tol=3e-2):
    C = _ext.native()
    q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, dtype, seed)
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    assert o.dtype == dtype and o.shape == (B, S, Hq, D) and lse.shape == (B, Hq, S)
    do = torch.randn(B, S, Hq, D, device=cuda).to(dtype)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal)
    o_r, lse_r, dq_r, dk_r, dv_r = oracle(q, k, v, do, causal, scale)
    assert _rel(o, o_r) < tol, _rel(o, o_r)
    assert (lse - lse_r).abs().max().item() < 2e-3
    for name, got, want in (("dq", dq, dq_r), ("dk", dk, dk_r), ("dv", dv, dv_r)):
        assert torch.isfinite(got.float()).all(), name
        # (S = 1: dq is exactly zero in exact math; compare absolutely against the scale of dk)
        err = _rel(got, want) if want.norm() > 1e-3 * dv_r.norm() else (got.float() - want).norm().item() / dv_r.norm().item()
        assert err < tol, (name, err)
    return q, k, v, o, lse, do, dq, dk, dv


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(2, 256, 4, 4, 128), (1, 512, 8, 2, 128), (1, 384, 4, 1, 64)])
@pytest.mark.parametrize("causal", [True, False])
def test_fp16_attention_fwd_bwd(cuda, B, S, Hq, Hkv, D, causal):
    _run(cuda, B, S, Hq, Hkv, D, causal, torch.float16, tol=1.5e-2)


@pytest.mark.parametrize("S", [1000, 130, 2047, 192, 1])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_untiled_seq_len(cuda, S, causal, dtype):
    _run(cuda, 2, S, 4, 2, 128 if S != 130 else 64, causal, dtype, seed=S)


@pytest.mark.parametrize("B,S,Hq,Hkv", [(1, 2048, 32, 32), (1, 8192, 32, 8)])
def test_production_shapes_default_kernels(cuda, attn_opts, B, S, Hq, Hkv):
    attn_opts(fwd_pipe=None, fwd_thr=None, dkdv_impl=None, dq_pipe=None, dkdv_split=None, dkdv_kreg=None)
    q, k, v, o, lse, do, dq, dk, dv = _run(cuda, B, S, Hq, Hkv, 128, True, torch.bfloat16, seed=7)
    # bit-reproducible backward at production shape (bit-exact resume relies on it)
    dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    _ext.native().attn_bwd(q, k, v, o, do, lse, dq2, dk2, dv2, 1 / math.sqrt(128), True)
    assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(2, 256, 4, 4, 128), (1, 512, 8, 2, 128), (1, 384, 4, 1, 64),
                                         (2, 1000, 4, 2, 128), (1, 130, 2, 1, 64), (2, 1, 4, 2, 128)])
@pytest.mark.parametrize("causal", [True, False])
def test_fp32_attention_fwd_bwd(cuda, B, S, Hq, Hkv, D, causal):
    """fp32 kernels (attention_f32.hip, v_mfma_f32_32x32x2_f32) against the fp32 oracle, incl.
    untiled lengths (zero-padded to 128 in the binding) and GQA; the backward is bit-reproducible."""
    q, k, v, o, lse, do, dq, dk, dv = _run(cuda, B, S, Hq, Hkv, D, causal, torch.float32, seed=S + D, tol=1e-4)
    dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    _ext.native().attn_bwd(q, k, v, o, do, lse, dq2, dk2, dv2, 1 / math.sqrt(D), causal)
    assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)


def test_flash_attention_op_fp32_hip_and_fp64_torch(cuda):
    """The autograd op: fp32 GPU tensors run the fp32 HIP kernels, fp64 the torch math."""
    for dt in (torch.float32, torch.float64):
        q, k, v = (t.clone().requires_grad_() for t in _qkv(cuda, 1, 100, 4, 2, 64, dt))
        o = F.flash_attention(q, k, v, causal=True)
        o.sum().backward()
        assert o.dtype == dt and q.grad.dtype == dt
        qd, kd, vd = (t.detach().double().requires_grad_() for t in (q, k, v))
        ref = R.attention_ref(qd, kd, vd, True)
        ref.sum().backward()
        tol = 1e-5 if dt == torch.float32 else 1e-10
        assert _rel(o.double(), ref) < tol
        for got, want in ((q.grad, qd.grad), (k.grad, kd.grad), (v.grad, vd.grad)):
            assert _rel(got.double(), want) < 10 * tol


def test_unsupported_head_dim_warns_once_and_stays_correct(cuda):
    """head_dim 96 is outside the MFMA kernels: the op runs torch math on the GPU, warns once (not
    silently 10x slower), and matches the oracle."""
    F._FALLBACK_WARNED.clear()
    q, k, v = _qkv(cuda, 1, 256, 4, 4, 96, torch.bfloat16)
    with pytest.warns(RuntimeWarning, match="attention .* runs PyTorch math"):
        o, _ = F._attn_fwd(q, k, v, 96 ** -0.5, True)
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("error")
        F._attn_fwd(q, k, v, 96 ** -0.5, True)  # the second call is silent
    ref_o = R.attention_ref(q.float(), k.float(), v.float(), True, 96 ** -0.5)
    assert _rel(o, ref_o) < 1e-2
