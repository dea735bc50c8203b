"""Numerics of every HIP kernel against a plain-PyTorch fp32 reference of the same op."""
import math

import pytest
import torch

from pyrecover_amd import _ext
from pyrecover_amd.ops import reference as R

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-6)).item()


# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("rows,D", [(333, 4096), (64, 768), (17, 128)])
@pytest.mark.parametrize("with_delta", [False, True])
def test_rmsnorm(cuda, rows, D, with_delta):
    C = _ext.native()
    torch.manual_seed(0)
    x = torch.randn(rows, D, device=cuda, dtype=torch.bfloat16)
    d = torch.randn(rows, D, device=cuda, dtype=torch.bfloat16) if with_delta else None
    w = (1 + 0.1 * torch.randn(D, device=cuda)).bfloat16()
    h, y, rstd = C.rmsnorm_fwd(x, d, w, 1e-5)
    h_ref = x if d is None else x + d
    y_ref = R.rmsnorm_ref(h_ref, w, 1e-5)
    assert torch.equal(h, h_ref)
    assert _rel(y, y_ref) < 1e-2
    # exact same rounding points as the reference in >99% of elements
    assert (y != y_ref).float().mean().item() < 0.01
    dy = torch.randn_like(x)
    dres = torch.randn_like(x) if with_delta else None
    dw = torch.empty_like(w)
    dx = C.rmsnorm_bwd(dy, h, w, rstd, dres, dw, False)
    # fp32 autograd oracle
    hf = h.float().requires_grad_()
    wf = w.float().requires_grad_()
    yf = (hf * torch.rsqrt(hf.pow(2).mean(-1, keepdim=True) + 1e-5)) * wf
    yf.backward(dy.float())
    gx = hf.grad + (dres.float() if dres is not None else 0)
    assert _rel(dx, gx) < 2e-2
    assert _rel(dw, wf.grad) < 2e-2
    # accumulate mode adds
    dw2 = dw.clone()
    C.rmsnorm_bwd(dy, h, w, rstd, dres, dw2, True)
    assert _rel(dw2, 2 * dw.float()) < 1e-2


@pytest.mark.parametrize("rows,D", [(333, 1024), (64, 768)])
@pytest.mark.parametrize("with_delta", [False, True])
def test_layernorm(cuda, rows, D, with_delta):
    C = _ext.native()
    torch.manual_seed(0)
    x = torch.randn(rows, D, device=cuda, dtype=torch.bfloat16)
    d = torch.randn(rows, D, device=cuda, dtype=torch.bfloat16) if with_delta else None
    w = (1 + 0.1 * torch.randn(D, device=cuda)).bfloat16()
    b = (0.1 * torch.randn(D, device=cuda)).bfloat16()
    h, y, mean, rstd = C.layernorm_fwd(x, d, w, b, 1e-5)
    h_ref = x if d is None else x + d
    hf = h_ref.float().requires_grad_()
    wf, bf = w.float().requires_grad_(), b.float().requires_grad_()
    yf = torch.nn.functional.layer_norm(hf, (D,), wf, bf, 1e-5)
    assert torch.equal(h, h_ref)
    assert _rel(y, yf) < 1e-2
    dy = torch.randn_like(x)
    dres = torch.randn_like(x) if with_delta else None
    yf.backward(dy.float())
    dwb = torch.empty(2 * D, device=cuda, dtype=torch.bfloat16)
    dx = C.layernorm_bwd(dy, h, w, mean, rstd, dres, dwb, False)
    gx = hf.grad + (dres.float() if dres is not None else 0)
    assert _rel(dx, gx) < 2e-2
    assert _rel(dwb[:D], wf.grad) < 2e-2 and _rel(dwb[D:], bf.grad) < 2e-2


def test_rope(cuda):
    C = _ext.native()
    B, S, Hq, Hkv, D = 2, 256, 4, 2, 128
    fc = R.precompute_freqs_cis(D, S, 500000.0)
    tab = R.rope_table(fc).to(cuda)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=cuda, dtype=torch.bfloat16)
    q = qkv[:, :Hq * D].view(B, S, Hq, D).clone()
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D).clone()
    v = qkv[:, (Hq + Hkv) * D:].clone()
    qr, kr = R.apply_rotary_emb_ref(q, k, fc.to(cuda))
    x = qkv.clone()
    C.rope_(x, (Hq + Hkv) * D, tab, D, S, 0, False)
    assert _rel(x[:, :Hq * D].view(B, S, Hq, D), qr) < 1e-2
    assert _rel(x[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D), kr) < 1e-2
    assert torch.equal(x[:, (Hq + Hkv) * D:], v)
    C.rope_(x, (Hq + Hkv) * D, tab, D, S, 0, True)  # inverse rotation restores
    assert _rel(x, qkv) < 2e-2


def test_swiglu(cuda):
    C = _ext.native()
    T, F = 300, 1024
    gu = torch.randn(T, 2 * F, device=cuda, dtype=torch.bfloat16)
    y = C.swiglu_fwd(gu)
    y_ref = R.swiglu_ref(gu[:, :F], gu[:, F:])
    assert _rel(y, y_ref) < 1e-2
    dy = torch.randn(T, F, device=cuda, dtype=torch.bfloat16)
    g = gu[:, :F].float().requires_grad_()
    u = gu[:, F:].float().requires_grad_()
    (torch.nn.functional.silu(g) * u).backward(dy.float())
    dgu = C.swiglu_bwd(dy, gu, None)
    assert _rel(dgu[:, :F], g.grad) < 2e-2
    assert _rel(dgu[:, F:], u.grad) < 2e-2


def test_embedding(cuda):
    C = _ext.native()
    V, D, T = 1000, 256, 4096
    W = torch.randn(V, D, device=cuda, dtype=torch.bfloat16)
    ids = torch.randint(0, V, (2, T // 2), device=cuda)
    out = C.embedding_fwd(ids, W)
    assert torch.equal(out, W[ids])
    dout = torch.randn(2, T // 2, D, device=cuda, dtype=torch.bfloat16)
    dW = torch.empty_like(W)
    C.embedding_bwd(ids, dout, dW, False)
    ref = torch.zeros(V, D, device=cuda).index_add_(0, ids.reshape(-1), dout.reshape(-1, D).float())
    assert _rel(dW, ref) < 1e-2
    dW2 = dW.clone()
    C.embedding_bwd(ids, dout, dW2, False)
    assert torch.equal(dW, dW2)  # deterministic


@pytest.mark.parametrize("V", [32000, 50304, 1000])
def test_cross_entropy(cuda, V):
    C = _ext.native()
    T = 257
    logits = (3 * torch.randn(T, V, device=cuda)).bfloat16()
    labels = torch.randint(0, V, (T,), device=cuda)
    labels[:13] = -100
    lse, loss_row, stats = C.xent_fwd(logits, labels, -100)
    ref = R.cross_entropy_ref(logits, labels)
    assert abs(stats[0].item() - ref.item()) < 1e-4 * max(1.0, ref.item())
    assert stats[1].item() == (labels != -100).sum().item()
    lf = logits.float().requires_grad_()
    R.cross_entropy_ref(lf, labels).backward()
    g = torch.full((1,), 0.5, device=cuda)
    d = logits.clone()
    C.xent_bwd_(d, labels, lse, stats, g, -100)
    assert _rel(d, 0.5 * lf.grad) < 2e-2
    assert d[:13].abs().max().item() == 0


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize("fast", [False, True])
def test_adamw_matches_torch_fused(cuda, fast, dtype):
    """The default kernel (fast=False) is bit-equal to torch's fused AdamW (the reference's
    --fused-optimizer) on p, m and v, including a tail that is not a multiple of 8; the opt-in
    hardware reciprocal / square root (fast=True) tracks it within a few fp32 ulps of p."""
    C = _ext.native()
    n = (1 << 22) + 5
    torch.manual_seed(1)
    p = torch.randn(n, device=cuda, dtype=dtype)
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    p2, m2, v2 = p.clone(), m.clone(), v.clone()
    step = torch.zeros((), device=cuda)
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.999, 1e-8, 0.01
    for s in range(1, 4):
        g = (torch.randn(n, device=cuda) * 10.0 ** (-s)).to(dtype)
        C.adamw_flat_(p, g, m, v, lr, b1, b2, eps, wd, 1 - b1 ** s, math.sqrt(1 - b2 ** s), 1.0, None, None, fast)
        step += 1
        torch._fused_adamw_([p2], [g], [m2], [v2], [], [step], amsgrad=False, lr=lr, beta1=b1, beta2=b2,
                            weight_decay=wd, eps=eps, maximize=False)
    if not fast:
        for a, b in ((p, p2), (m, m2), (v, v2)):
            bad = (a != b).nonzero()
            assert bad.numel() == 0, (bad.numel(), bad[:4].flatten().tolist(), a[bad[:4, 0]].tolist(),
                                      b[bad[:4, 0]].tolist())
    elif dtype != torch.float32:  # a few fp32 ulps of p rarely survive the 16-bit rounding
        assert (p != p2).float().mean().item() < 1e-3
    assert _rel(p, p2) < 1e-2 and _rel(m, m2) < 1e-2 and _rel(v, v2) < 1e-2


@pytest.mark.parametrize("n", [(1 << 22) + 5, 1000])
def test_adamw_master_matches_fp32_torch_fused(cuda, n):
    """--master-weights fp32: the fp32 master, m and v are bit-equal to torch's fused AdamW run in fp32
    on the widened bf16 gradient, and the bf16 parameter is the master rounded to nearest even (the
    odd n exercises the scalar tail)."""
    C = _ext.native()
    torch.manual_seed(2)
    pm = torch.randn(n, device=cuda)
    p = pm.to(torch.bfloat16)
    m = torch.zeros_like(pm)
    v = torch.zeros_like(pm)
    p2, m2, v2 = pm.clone(), m.clone(), v.clone()
    step = torch.zeros((), device=cuda)
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.95, 1e-8, 0.1
    for s in range(1, 4):
        g = (torch.randn(n, device=cuda) * 10.0 ** (-s)).to(torch.bfloat16)
        C.adamw_master_(p, pm, g, m, v, lr, b1, b2, eps, wd, 1 - b1 ** s, math.sqrt(1 - b2 ** s), 1.0)
        step += 1
        torch._fused_adamw_([p2], [g.float()], [m2], [v2], [], [step], amsgrad=False, lr=lr, beta1=b1, beta2=b2,
                            weight_decay=wd, eps=eps, maximize=False)
    assert torch.equal(pm, p2) and torch.equal(m, m2) and torch.equal(v, v2)
    assert torch.equal(p, p2.to(torch.bfloat16))


def test_grad_norm(cuda):
    C = _ext.native()
    x = torch.randn(3_000_001, device=cuda, dtype=torch.bfloat16)
    out = C.grad_norm(x, 1.0, 1.0)
    ref = x.float().norm()
    assert abs(out[0].item() - ref.item()) < 1e-3 * ref.item()
    assert abs(out[1].item() - min(1.0, 1.0 / (ref.item() + 1e-6))) < 1e-5


# ------------------------------------------------------------------------------------------
def _qkv(cuda, B, S, Hq, Hkv, D, seed=0, scale=1.0):
    torch.manual_seed(seed)
    qkv = (scale * torch.randn(B * S, (Hq + 2 * Hkv) * D, device=cuda)).bfloat16()
    q = qkv[:, :Hq * D].view(B, S, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(B, S, Hkv, D)
    return qkv, q, k, v


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 256, 4, 4, 128), (2, 512, 8, 2, 128), (1, 384, 4, 1, 64),
                                          (1, 128, 2, 2, 64), (1, 192, 4, 2, 128)])
@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("pipe", [0, 1])
def test_attention_fwd(cuda, attn_opts, pipe, B, S, Hq, Hkv, D, causal):
    """Every forward kernel (fwd_pipe: fwd_kernel / cross-tile pipelined fwd_p_kernel)."""
    attn_opts(fwd_pipe=pipe)
    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D)
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    o_ref, lse_ref = R.attention_lse_ref(q, k, v, causal, scale)
    assert (o.float() - o_ref).abs().max().item() < 2e-2
    assert (lse - lse_ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal", [(4, 512, 8, 8, 128, True), (2, 1024, 16, 4, 128, True),
                                                 (2, 768, 16, 4, 64, False)])
@pytest.mark.parametrize("kreg", [-2, 0])
def test_attention_block_order_is_bitwise_neutral(cuda, attn_opts, kreg, B, S, Hq, Hkv, D, causal):
    """The XCD-grouped block order (fwd_order / dq_order / dkdv_order) only changes which workgroup
    computes which tile: every setting gives the same bits as the heavy-first order, forward and
    backward (ring and LDS dK/dV kernels), and matches the fp32 oracle."""
    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=7)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    scale = 1 / math.sqrt(D)
    outs = {}
    cases = [0, 1, 2, 4, -1]
    for order in cases:
        attn_opts(fwd_order=order, dq_order=order, dkdv_order=order, dkdv_kreg=kreg)
        o, lse = C.attn_fwd(q, k, v, scale, causal)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal)
        outs[order] = (o, lse, dq, dk, dv)
    for case in cases[1:]:
        assert all(torch.equal(a, b) for a, b in zip(outs[0], outs[case])), case
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    o, _, dq, dk, dv = outs[-1]
    assert (o.float() - of).abs().max().item() < 2e-2
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert _rel(got, want) < 3e-2, (_rel(got, want))


@pytest.mark.parametrize("pipe", [0, 1])
@pytest.mark.parametrize("thr", [0.0, 8.0])
def test_attention_fwd_rescale_spike(cuda, attn_opts, pipe, thr):
    """Forces the online-softmax running max to jump at a late key tile (rule 26), with the exact
    rescale (fwd_thr=0) and the default deferred threshold."""
    attn_opts(fwd_pipe=pipe, fwd_thr=thr)
    C = _ext.native()
    B, S, H, D = 1, 512, 2, 128
    _, q, k, v = _qkv(cuda, B, S, H, H, D, seed=3)
    k = k.clone()
    q = q.clone()
    q[0, 400, 0] = 4.0
    k[0, 390, 0] = 4.0  # huge score for query 400 at key tile 6
    o, lse = C.attn_fwd(q, k, v, 1 / math.sqrt(D), True)
    o_ref, lse_ref = R.attention_lse_ref(q, k, v, True, 1 / math.sqrt(D))
    assert (o.float() - o_ref).abs().max().item() < 2e-2
    assert (lse - lse_ref).abs().max().item() < 1e-3


@pytest.mark.parametrize("B,S,Hq,Hkv,D", [(1, 256, 4, 4, 128), (2, 256, 8, 2, 128), (1, 384, 4, 1, 64),
                                          (1, 128, 2, 2, 64)])
@pytest.mark.parametrize("causal", [True, False])
def test_attention_bwd(cuda, B, S, Hq, Hkv, D, causal):
    C = _ext.native()
    qkv, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=1)
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    dqkv = torch.zeros_like(qkv)
    nq, nk = Hq * D, Hkv * D
    dq = dqkv[:, :nq].view(B, S, Hq, D)
    dk = dqkv[:, nq:nq + nk].view(B, S, Hkv, D)
    dv = dqkv[:, nq + nk:].view(B, S, Hkv, D)
    C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert _rel(got, want) < 3e-2, (_rel(got, want))
    # deterministic: identical bits on a second run
    dqkv2 = torch.zeros_like(qkv)
    C.attn_bwd(q, k, v, o, do, lse, dqkv2[:, :nq].view(B, S, Hq, D), dqkv2[:, nq:nq + nk].view(B, S, Hkv, D),
               dqkv2[:, nq + nk:].view(B, S, Hkv, D), scale, causal)
    assert torch.equal(dqkv, dqkv2)


@pytest.mark.parametrize("impl", [0, 1, 2, 3])
@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal", [(1, 1024, 4, 1, 128, True), (2, 512, 4, 2, 128, False),
                                                 (1, 640, 2, 2, 64, True)])
def test_attention_bwd_dkdv_kernels(cuda, attn_opts, impl, B, S, Hq, Hkv, D, causal):
    """Every backward kernel generation -- dK/dV two-wave vs one-wave-per-SIMD pipelined
    (dkdv_impl), dQ plain vs region-pipelined (dq_pipe) -- against the fp32 oracle, with
    multi-step loops, GQA and the causal diagonal. impl 2: the two-wave kernel with K held in
    registers (dkdv_kreg 1; 256-key blocks at D = 128); impl 3: the ring-staged two-wave kernel
    (dkdv_kreg 2, the default: K in registers, Q/dO/row constants by LDS-DMA), bitwise equal to the
    LDS-K kernel."""
    kreg = {0: 0, 1: 0, 2: 1, 3: 2}[impl]
    attn_opts(dkdv_impl=min(impl, 1) if impl < 2 else 0, dq_pipe=min(impl, 1), dkdv_kreg=kreg)
    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=5)
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    for got, want in ((dq, qf.grad), (dk, kf.grad), (dv, vf.grad)):
        assert _rel(got, want) < 3e-2, (_rel(got, want))
    dq2, dk2, dv2 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq2, dk2, dv2, scale, causal)
    assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)
    if impl >= 2:  # K in registers reads the same values as K from LDS: bitwise the same gradients
        attn_opts(dkdv_kreg=0)
        C.attn_bwd(q, k, v, o, do, lse, dq2, dk2, dv2, scale, causal)
        assert torch.equal(dq, dq2) and torch.equal(dk, dk2) and torch.equal(dv, dv2)


@pytest.mark.parametrize("split", [2, 4])
@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal,rope", [(1, 1024, 8, 2, 128, True, True), (2, 512, 4, 1, 128, False, False),
                                                      (1, 640, 4, 1, 64, True, True)])
def test_attention_bwd_dkdv_query_head_split(cuda, attn_opts, split, B, S, Hq, Hkv, D, causal, rope):
    """The pipelined dK/dV kernel with the kv head's query heads split over blocks (fp32 parts plus the
    reduction pass, the small-batch GQA path): against the fp32 oracle and the unsplit kernel, with the
    fused inverse RoPE on dK, and deterministic run to run."""
    from pyrecover_amd.ops.reference import precompute_freqs_cis, rope_table

    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=11)
    scale = 1 / math.sqrt(D)
    tab = rope_table(precompute_freqs_cis(D, S, 10000.0)).to(cuda) if rope else None
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    res = {}
    for n in (1, split, split):
        attn_opts(dkdv_impl=1, dkdv_split=n)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal, tab)
        if n in res:
            assert all(torch.equal(a, b) for a, b in zip(res[n], (dq, dk, dv)))
        res[n] = (dq, dk, dv)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    dk32 = kf.grad
    if rope:
        dk32 = dk32.reshape(B * S, Hkv * D).clone()
        R.rope_inplace_2d(dk32, Hkv * D, tab, D, S, inverse=True)
        dk32 = dk32.view(B, S, Hkv, D)
    # by grid (-1): split without a window job, unsplit when a side-stream job waits for the dK/dV
    # window (mid_event)
    attn_opts(dkdv_impl=1, dkdv_split=-1)
    for with_event in (False, True):
        ev = torch.cuda.Event()
        ev.record()
        d3 = [torch.empty_like(t) for t in (q, k, v)]
        C.attn_bwd(q, k, v, o, do, lse, *d3, scale, causal, tab, ev.cuda_event if with_event else 0)
        torch.cuda.synchronize()
        n, grid = 1, (S // 128) * Hkv * B  # attention.hip dkdv_split(): the by-grid choice
        while grid * n < (512 if D == 128 else 1024) and (Hq // Hkv) % (2 * n) == 0:
            n *= 2
        want = res[1] if with_event else res.get(n)
        if want is not None:
            assert all(torch.equal(a, b) for a, b in zip(d3, want)), with_event
    dq, dk, dv = res[split]
    assert torch.equal(dq, res[1][0])  # the dQ kernel is not split
    for got, want in ((dk, dk32), (dv, vf.grad)):
        assert _rel(got, want) < 3e-2, _rel(got, want)
    for got, base in ((dk, res[1][1]), (dv, res[1][2])):
        assert _rel(got, base.float()) < 1e-2


@pytest.mark.parametrize("impl", [0, 1])
@pytest.mark.parametrize("B,S,Hq,Hkv,D,causal", [(2, 512, 8, 2, 128, True), (1, 384, 4, 1, 64, True),
                                                 (1, 256, 4, 4, 128, False), (1, 1000, 4, 2, 128, True)])
def test_attention_bwd_fused_inverse_rope(cuda, attn_opts, impl, B, S, Hq, Hkv, D, causal):
    """attn_bwd(..., rope_tab): dq / dk leave the kernels with the inverse RoPE applied (fp32, rounded
    once) -- against the fp32 oracle of the unfused op (backward + inverse rotation), for both dK/dV
    kernels, GQA, D = 64 and a padded (untiled) sequence; dv is bitwise the unfused one."""
    from pyrecover_amd.ops.reference import precompute_freqs_cis, rope_table

    attn_opts(dkdv_impl=impl, dq_pipe=impl)
    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=9)
    scale = 1 / math.sqrt(D)
    tab = rope_table(precompute_freqs_cis(D, S + 64, 10000.0)).to(cuda)  # longer table: rows = positions
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal, tab)
    dq0, dk0, dv0 = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq0, dk0, dv0, scale, causal)
    assert torch.equal(dv, dv0)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    for got, g32, H in ((dq, qf.grad, Hq), (dk, kf.grad, Hkv)):
        want = g32.reshape(B * S, H * D).clone()
        R.rope_inplace_2d(want, H * D, tab, D, S, inverse=True)
        assert _rel(got, want.view(B, S, H, D)) < 3e-2, _rel(got, want.view(B, S, H, D))
    # identical to the separate inverse-RoPE pass up to one bf16 rounding of the unrotated values
    for got, base, H in ((dq, dq0, Hq), (dk, dk0, Hkv)):
        sep = base.reshape(B * S, H * D).clone()
        C.rope_(sep, H * D, tab, D, S, 0, True)
        assert _rel(got, sep.view(B, S, H, D).float()) < 1e-2


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,rope", [(1, 1024, 4, 1, True, True), (2, 512, 4, 2, False, True),
                                                    (2, 768, 3, 3, True, False), (1, 256, 2, 2, False, False)])
def test_attention_bwd_fused_kernel(cuda, attn_opts, B, S, Hq, Hkv, causal, rope):
    """attention_bwd_fused.hip (dQ, dK, dV of a (batch, kv head) in one workgroup; dQ summed over the
    key blocks in order through an fp32 workspace): against the fp32 oracle (with the inverse RoPE on
    dq / dk), multi-block causal and full attention, GQA; bitwise deterministic run to run; dV bitwise
    equal to the split ring-staged dK/dV kernel (same P)."""
    from pyrecover_amd.ops.reference import precompute_freqs_cis, rope_table

    D = 128
    C = _ext.native()
    _, q, k, v = _qkv(cuda, B, S, Hq, Hkv, D, seed=13)
    scale = 1 / math.sqrt(D)
    tab = rope_table(precompute_freqs_cis(D, S, 10000.0)).to(cuda) if rope else None
    o, lse = C.attn_fwd(q, k, v, scale, causal)
    do = torch.randn(B, S, Hq, D, device=cuda).bfloat16()
    outs = []
    for fused in (1, 1, 0):
        attn_opts(bwd_fused=fused, dkdv_kreg=2, dkdv_impl=0)
        d3 = [torch.full_like(t, float("nan")) for t in (q, k, v)]
        C.attn_bwd(q, k, v, o, do, lse, *d3, scale, causal, tab)
        outs.append(d3)
    (dq, dk, dv), again, split = outs
    assert all(torch.equal(a, b) for a, b in zip((dq, dk, dv), again))
    assert torch.equal(dv, split[2])
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of, _ = R.attention_lse_ref(qf, kf, vf, causal, scale)
    of.backward(do.float())
    for got, g32, H in ((dq, qf.grad, Hq), (dk, kf.grad, Hkv), (dv, vf.grad, Hkv)):
        want = g32
        if rope and got is not dv:
            want = g32.reshape(B * S, H * D).clone()
            R.rope_inplace_2d(want, H * D, tab, D, S, inverse=True)
            want = want.view(B, S, H, D)
        assert torch.isfinite(got.float()).all()
        assert _rel(got, want) < 3e-2, _rel(got, want)
    for got, base in zip((dq, dk), split[:2]):
        assert _rel(got, base.float()) < 1e-2


@pytest.mark.parametrize("T,F,dtype", [(4096, 1024, torch.bfloat16), (1000, 392, torch.bfloat16),
                                       (512, 256, torch.float16), (256, 136, torch.float32)])
def test_swiglu_bwd_variants_bitwise(cuda, T, F, dtype):
    """The hoisted tile kernels (4 and 8 tokens per lane, partial row / column tiles) equal the
    grid-stride kernel bit for bit, in place over gu and out of place."""
    C_ = _ext.native()
    torch.manual_seed(T + F)
    gu = torch.randn(T, 2 * F, device=cuda).to(dtype)
    dy = torch.randn(T, F, device=cuda).to(dtype)
    ref = C_.swiglu_bwd(dy, gu, None, 0)
    for var in (1, 2, -1):
        assert torch.equal(C_.swiglu_bwd(dy, gu, None, var), ref)
        g2 = gu.clone()
        C_.swiglu_bwd(dy, g2, g2, var)
        assert torch.equal(g2, ref)


def test_single_hip_runtime_loaded(cuda):
    """The extension must bind to torch's HIP runtime, not load a second copy."""
    maps = open("/proc/self/maps").read()
    libs = {line.split()[-1] for line in maps.splitlines() if "libamdhip64" in line}
    assert len(libs) == 1, libs


@pytest.mark.parametrize("R,C", [(64, 64), (256, 192), (2048, 1024), (128, 32000)])
def test_transpose2d_exact(cuda, R, C):
    C_ = _ext.native()
    x = torch.randn(R, C, device=cuda).bfloat16()
    assert torch.equal(C_.transpose2d(x), x.t().contiguous())
    xs = torch.randn(R, C + 64, device=cuda).bfloat16()[:, 64:]  # strided rows
    assert torch.equal(C_.transpose2d(xs), xs.t().contiguous())


@pytest.mark.parametrize("T,F,dtype", [(256, 192, torch.bfloat16), (64, 192, torch.bfloat16),
                                       (2048, 1024, torch.bfloat16), (128, 256, torch.float16)])
def test_swiglu_bwd_t_matches_swiglu_bwd_exactly(cuda, T, F, dtype):
    # two-tile kernel (F % 128 == 0) and its one-tile fallback (F = 192) against the row-major kernel
    C_ = _ext.native()
    gu = torch.randn(T, 2 * F, device=cuda).to(dtype)
    dy = torch.randn(T, F, device=cuda).to(dtype)
    ref = C_.swiglu_bwd(dy, gu.clone(), None)
    g2 = gu.clone()
    guT = C_.swiglu_bwd_t_(dy, g2)
    assert torch.equal(g2, ref)
    assert torch.equal(guT, ref.t().contiguous())


@pytest.mark.parametrize("T,F", [(256, 192), (64, 192), (2048, 1024)])
def test_swiglu_fwd_t_matches_swiglu_fwd_exactly(cuda, T, F):
    C_ = _ext.native()
    gu = torch.randn(T, 2 * F, device=cuda).bfloat16()
    ref = C_.swiglu_fwd(gu)
    a, aT = C_.swiglu_fwd_t(gu)
    assert torch.equal(a, ref)
    assert torch.equal(aT, ref.t().contiguous())


def test_attention_bwd_delta_many_heads(cuda):
    """delta = rowsum(dO * O) (computed by the dQ kernel) with a head count that is not a power of
    two and D = 64: dq/dk/dv against the fp32 oracle."""
    C = _ext.native()
    B, S, Hq, Hkv, D = 1, 128, 12, 12, 64
    q, k, v = (torch.randn(B, S, H, D, device=cuda).bfloat16() for H in (Hq, Hkv, Hkv))
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn_like(o)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True)
    qf, kf, vf = (t.float().requires_grad_() for t in (q, k, v))
    of = R.attention_ref(qf, kf, vf, causal=True, scale=scale)
    of.backward(do.float())
    assert _rel(dq, qf.grad) < 2e-2
    assert _rel(dk, kf.grad) < 2e-2
    assert _rel(dv, vf.grad) < 2e-2


def test_rope_t_matches_rope_exactly(cuda):
    from pyrecover_amd.ops.reference import precompute_freqs_cis, rope_table

    C_ = _ext.native()
    B, S, Hq, Hkv, D = 2, 128, 4, 2, 64
    tab = rope_table(precompute_freqs_cis(D, S, 10000.0)).to(cuda)
    x = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=cuda).bfloat16()
    ref = x.clone()
    C_.rope_(ref, (Hq + Hkv) * D, tab, D, S, 0, True)
    x2 = x.clone()
    xT = C_.rope_t_(x2, (Hq + Hkv) * D, tab, D, S, True)
    assert torch.equal(x2, ref)
    assert torch.equal(xT, ref.t().contiguous())


@pytest.mark.parametrize("rows,cols", [(64, 64), (192, 320), (4096, 128), (128, 512), (256, 384), (384, 1152)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("fast", [False, True])
def test_adamw_t_matches_flat_adamw_plus_transpose(cuda, rows, cols, dtype, fast):
    """Fused AdamW + transposed-shadow write == flat AdamW followed by transpose2d, bit for bit
    (incl. device-side grad scale and hyper-parameters), with 128 x 128 tiles and the 64 x 64
    fallback (a dim that is not a multiple of 128)."""
    C = _ext.native()
    torch.manual_seed(rows + cols)
    p = torch.randn(rows, cols, device=cuda).to(dtype)
    g = (torch.randn(rows, cols, device=cuda) * 1e-2).to(dtype)
    m = (torch.randn(rows, cols, device=cuda) * 1e-3).to(dtype)
    v = (torch.rand(rows, cols, device=cuda) * 1e-4).to(dtype)
    gs = torch.tensor([0.7], device=cuda)
    hy = torch.tensor([3e-4, 0.19, 0.031], device=cuda, dtype=torch.float64)
    a = [t.clone() for t in (p, g, m, v)]
    C.adamw_flat_(a[0].view(-1), a[1].view(-1), a[2].view(-1), a[3].view(-1), 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.2,
                  0.5, gs, hy, fast)
    pt_ref = C.transpose2d(a[0])
    b = [t.clone() for t in (p, g, m, v)]
    pt = torch.empty(cols, rows, device=cuda, dtype=dtype)
    C.adamw_t_(b[0], b[1], b[2], b[3], pt, 1e-3, 0.9, 0.95, 1e-8, 0.1, 0.5, 0.2, 0.5, gs, hy, fast)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert torch.equal(pt, pt_ref)


# ---------------------------------------------------------------------------------------
# Weight-gradient MFMA GEMM (csrc/kernels/gemm_wgrad.hip): out (+)= a^T b on row-major operands
@pytest.mark.parametrize("K,M,N,dtype", [(32, 256, 256, torch.bfloat16), (2048, 768, 512, torch.bfloat16),
                                         (4096, 512, 1024, torch.float16), (96, 1280, 256, torch.bfloat16),
                                         # 300 tiles on 256 CUs: 44 tail tiles split over K
                                         (1024, 7680, 2560, torch.bfloat16)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_wgrad_mm_vs_fp32(cuda, K, M, N, dtype, accumulate):
    C_ = _ext.native()
    g = torch.Generator(device=cuda)
    g.manual_seed(K + M + N)
    a = torch.randn(K, M, device=cuda, generator=g).to(dtype)
    b = torch.randn(K, N, device=cuda, generator=g).to(dtype)
    c0 = torch.randn(M, N, device=cuda, generator=g).to(dtype)
    out = c0.clone()
    C_.wgrad_mm_(a, b, out, accumulate)
    ref = a.double().t() @ b.double() + (c0.double() if accumulate else 0)
    # one rounding of the fp32 result to the 16-bit output
    err = ((out.double() - ref).abs() / (ref.abs() + math.sqrt(K))).max().item()
    assert err < (1e-2 if dtype == torch.bfloat16 else 2e-3), err
    out2 = c0.clone()
    C_.wgrad_mm_(a, b, out2, accumulate)
    assert torch.equal(out, out2)  # deterministic


@pytest.mark.parametrize("M,N", [(12288, 4096), (4096, 4096), (22016, 4096), (4096, 11008), (32000, 4096)])
def test_wgrad_mm_production_shapes_k32768(cuda, M, N):
    """The 7B B16 step's weight gradients (QKV, O, W1|W3, W2, head) at K = 32768 tokens, default
    split settings, against an fp32 oracle."""
    C_ = _ext.native()
    K = 32768
    g = torch.Generator(device=cuda)
    g.manual_seed(M + N)
    a = ((torch.rand(K, M, device=cuda, generator=g) * 2 - 1) * 0.1).bfloat16()
    b = ((torch.rand(K, N, device=cuda, generator=g) * 2 - 1)).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    C_.wgrad_mm_(a, b, out, False)
    ref = torch.mm(a.float().t(), b.float())
    err = (out.float() - ref).abs()
    assert (err <= ref.abs() * 2 ** -8 + 1e-3).all().item(), err.max().item()


def test_wgrad_mm_strided_rows_and_slot_views(cuda):
    """Operands that are column slices of wider activations (row stride > width) and an output
    that is a view into a larger flat buffer, as the flat gradient slots are."""
    C_ = _ext.native()
    torch.manual_seed(3)
    big_a = torch.randn(512, 1024 + 256, device=cuda).bfloat16()
    big_b = torch.randn(512, 512 + 64, device=cuda).bfloat16()
    a, b = big_a[:, 256:], big_b[:, 64:]
    flat = torch.zeros(1024 * 512 + 4096, device=cuda, dtype=torch.bfloat16)
    out = flat[4096:].view(1024, 512)
    C_.wgrad_mm_(a, b, out, False)
    ref = a.float().t() @ b.float()
    assert ((out.float() - ref).norm() / ref.norm()).item() < 5e-3
    assert flat[:4096].abs().sum().item() == 0


def test_wgrad_mm_rejects_bad_shapes(cuda):
    C_ = _ext.native()
    a = torch.randn(64, 300, device=cuda).bfloat16()
    b = torch.randn(64, 256, device=cuda).bfloat16()
    with pytest.raises(RuntimeError):
        C_.wgrad_mm_(a, b, torch.empty(300, 256, device=cuda, dtype=torch.bfloat16), False)


def test_wgrad_mm_split_tail_under_hip_graph_capture(cuda):
    """The split tail's ticket memset and workspace are captured into a HIP graph (train.py
    --compile); replays are bit-identical to eager calls, including after the inputs change."""
    C_ = _ext.native()
    torch.manual_seed(5)
    K, M, N = 1024, 7680, 2560  # 300 tiles: 44 tail tiles split over K
    a = torch.randn(K, M, device=cuda).bfloat16()
    b = torch.randn(K, N, device=cuda).bfloat16()
    out = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        C_.wgrad_mm_(a, b, out, False)  # warm-up outside capture
    torch.cuda.current_stream(cuda).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        C_.wgrad_mm_(a, b, out, False)
    for _ in range(2):
        a.copy_(torch.randn(K, M, device=cuda).bfloat16())
        g.replay()
        torch.cuda.synchronize()
        ref = torch.empty_like(out)
        C_.wgrad_mm_(a, b, ref, False)
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
    exact = a.float().t() @ b.float()
    assert ((out.float() - exact).norm() / exact.norm()).item() < 5e-3


