"""Public module API parity: Attention / FeedForward / TransformerBlock forwards with the
reference's call signatures (reference model.py:194-230, 268-269, 325-327), checked against an
explicit composition of the reference's math (fp32, CPU) for outputs and parameter gradients.
A GPU variant runs the same modules on the HIP kernels in bf16."""
import pytest
import torch

from pyrecover_amd.config import get_preset
from pyrecover_amd.models.llama import Attention, FeedForward, Transformer, TransformerBlock
from pyrecover_amd.ops import reference as R


def ref_attention(at, x, freqs_cis):
    B, S, _ = x.shape
    q = (x @ at.wq.weight.t()).view(B, S, at.n_heads, at.head_dim)
    k = (x @ at.wk.weight.t()).view(B, S, at.n_kv_heads, at.head_dim)
    v = (x @ at.wv.weight.t()).view(B, S, at.n_kv_heads, at.head_dim)
    q, k = R.apply_rotary_emb_ref(q, k, freqs_cis)
    return R.attention_ref(q, k, v, True).reshape(B, S, -1) @ at.wo.weight.t()


def ref_ff(ff, x):
    return R.swiglu_ref(x @ ff.w1.weight.t(), x @ ff.w3.weight.t()) @ ff.w2.weight.t()


def ref_block(L, x, freqs_cis):
    h = x + ref_attention(L.attention, R.rmsnorm_ref(x, L.attention_norm.weight, L.attention_norm.eps), freqs_cis)
    return h + ref_ff(L.feed_forward, R.rmsnorm_ref(h, L.ffn_norm.weight, L.ffn_norm.eps))


def _check(mod, fn_fused, fn_ref, x, tol):
    x1 = x.clone().requires_grad_()
    y = fn_fused(mod, x1)
    g = torch.randn_like(y)
    y.backward(g)
    got = {n: p.grad.float().cpu().clone() for n, p in mod.named_parameters()}
    dx = x1.grad.float().cpu()
    mod.zero_grad(set_to_none=True)
    ref = mod.float().cpu() if x.is_cuda else mod
    xr = x.detach().float().cpu().requires_grad_()
    yr = fn_ref(ref, xr)
    yr.backward(g.float().cpu())

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()

    assert rel(y.detach().float().cpu(), yr.detach()) < tol
    assert rel(dx, xr.grad) < tol
    for n, p in ref.named_parameters():
        assert rel(got[n], p.grad) < tol, n


@pytest.mark.parametrize("kv", [None, 2])
def test_module_forwards_match_reference_math(kv):
    torch.manual_seed(0)
    a = get_preset("llama-micro", seq_len=64, n_kv_heads=kv)
    m = Transformer(a)
    fc = m.freqs_cis
    x = torch.randn(2, 48, a.dim)  # S below the model's seq_len: freqs_cis is sliced like the reference's
    _check(m.layers["0"].attention, lambda mod, t: mod(t, fc), lambda mod, t: ref_attention(mod, t, fc), x, 1e-4)
    _check(m.layers["0"].feed_forward, lambda mod, t: mod(t), ref_ff, x, 1e-4)
    _check(m.layers["1"], lambda mod, t: mod(t, fc), lambda mod, t: ref_block(mod, t, fc), x, 1e-4)


def test_modules_construct_standalone():
    a = get_preset("llama-micro", seq_len=32)
    at = Attention(a)
    ff = FeedForward(a.dim, 4 * a.dim, a.multiple_of, a.ffn_dim_multiplier)
    blk = TransformerBlock(0, a)
    fc = R.precompute_freqs_cis(a.dim // a.n_heads, a.seq_len, a.rope_theta)
    x = torch.randn(1, 32, a.dim)
    assert at(x, fc).shape == x.shape and ff(x).shape == x.shape and blk(x, fc).shape == x.shape


@pytest.mark.gpu
def test_module_forwards_on_gpu(cuda):
    torch.manual_seed(0)
    a = get_preset("llama-tiny", seq_len=256, n_kv_heads=2)
    m = Transformer(a).to(cuda, torch.bfloat16)
    fc = m.freqs_cis
    x = torch.randn(2, 256, a.dim, device=cuda, dtype=torch.bfloat16)
    _check(m.layers["0"].attention, lambda mod, t: mod(t, fc), lambda mod, t: ref_attention(mod, t, fc.cpu()), x, 3e-2)
    _check(m.layers["0"].feed_forward.to(cuda, torch.bfloat16), lambda mod, t: mod(t), ref_ff, x, 3e-2)
    _check(m.layers["1"].to(cuda, torch.bfloat16), lambda mod, t: mod(t, fc),
           lambda mod, t: ref_block(mod, t, fc.cpu()), x, 3e-2)


def test_wgrad_site_selection_parsing():
    """PYRECOVER_WGRAD: named sets, comma lists of sites, unknown sites rejected; the CPU path
    never selects the HIP weight-gradient kernel."""
    import pytest
    import torch

    from pyrecover_amd.ops import fused

    assert fused._wgrad_sites("lib") == frozenset()
    assert fused._wgrad_sites("auto") == frozenset({"qkv", "o", "w13", "head"})
    assert fused._wgrad_sites("hip") == frozenset({"qkv", "o", "w13", "w2", "head"})
    assert fused._wgrad_sites("o, qkv") == frozenset({"o", "qkv"})
    with pytest.raises(ValueError):
        fused._wgrad_sites("o,attn")
    x = torch.zeros(32768, 256, dtype=torch.bfloat16)
    assert not fused._hip_wgrad_ok(x, x, "o")


def test_wgrad_auto_needs_one_tile_per_cu(monkeypatch):
    """auto mode sends weight gradients with fewer 256 x 256 output tiles than CUs (GPT-2-medium)
    to the library; the 7B shapes keep the MFMA kernel."""
    import torch

    from pyrecover_amd.ops import fused

    monkeypatch.setattr(fused, "_cus", lambda t: 256)
    t = torch.zeros(1)
    assert not fused._wgrad_fills_chip(t, (3072, 1024))  # GPT-2-medium QKV: 48 tiles
    assert not fused._wgrad_fills_chip(t, (5632, 1024))  # GPT-2-medium W1|W3: 88 tiles
    assert fused._wgrad_fills_chip(t, (4096, 4096))  # 7B O: 256 tiles
    assert fused._wgrad_fills_chip(t, (22016, 4096))  # 7B W1|W3: 1376 tiles


def test_weight_shadow_site_policy(monkeypatch):
    """PRA_WEIGHT_SHADOWS: auto (none for a grouped-query model at <= 4096 tokens per step, every
    site otherwise: profiles/r6/shadows/), 1 / 0 and site lists; unknown sites are refused."""
    monkeypatch.delenv("PRA_WEIGHT_SHADOWS", raising=False)
    assert Transformer.shadow_sites("1") == Transformer.SHADOW_SITES
    assert Transformer.shadow_sites(False) == ()
    assert Transformer.shadow_sites("o, w2") == ("o", "w2")
    with pytest.raises(ValueError):
        Transformer.shadow_sites("qkv,mlp")

    def sites(tokens, **over):
        return Transformer(get_preset("llama-tiny", seq_len=64, **over)).flatten_(tokens_per_step=tokens).shadow_sites

    assert sites(2048, n_kv_heads=2) == ()  # GQA at 2048 tokens (Llama-3-8B S2048 B1)
    assert sites(8192, n_kv_heads=2) == Transformer.SHADOW_SITES  # GQA at 8192 tokens
    assert sites(2048, n_kv_heads=4) == Transformer.SHADOW_SITES  # MHA (Llama-2-7B B1)
    monkeypatch.setenv("PRA_WEIGHT_SHADOWS", "w13,head")
    flat = Transformer(get_preset("llama-tiny", seq_len=64, n_kv_heads=2)).flatten_(tokens_per_step=2048)
    assert flat.shadow_sites == ("w13", "head")  # (shadows themselves exist only for 16-bit GPU buffers)


def test_fused_attention_backward_env_selects_by_shape(monkeypatch):
    """PYRECOVER_ATTN_BWD_FUSED=1 means the fused backward where its grid fills the chip (launcher
    mode -1), so a batch-1 job never runs it; 0 keeps the split kernels."""
    from pyrecover_amd import _ext

    monkeypatch.setenv("PYRECOVER_ATTN_BWD_FUSED", "1")
    assert _ext._attn_env() == {"bwd_fused": -1}
    monkeypatch.setenv("PYRECOVER_ATTN_BWD_FUSED", "0")
    assert _ext._attn_env() == {"bwd_fused": 0}
