"""Fused autograd ops of the Transformer hot path.

Each op runs the HIP kernels of ``pyrecover_amd._C`` for GPU tensors and the plain-torch math of
:mod:`pyrecover_amd.ops.reference` for CPU tensors (CPU/gloo runs only). GEMMs run on the
hand-written MFMA kernels (csrc/kernels/gemm_nt.hip for forward / data gradients, with RoPE and
SwiGLU fused into their epilogues; gemm_wgrad.hip for weight gradients) wherever their shape rules
and the site selection allow, else on the library (``torch.mm`` -> hipBLASLt).

Weight gradients are produced directly into *gradient slots* (:mod:`pyrecover_amd.parallel.flat`)
instead of being returned to autograd, so they land in the flat gradient buffer / DDP bucket
without an AccumulateGrad pass. The parameters are still passed as inputs so autograd knows the
graph depends on them; their returned gradient is ``None``.

Reference parity (reference model.py): embedding (:355,388), RMSNorm (:25-49) with the residual
adds of TransformerBlock.forward (:325-327), Attention.forward (:194-230: QKV projections, RoPE,
causal SDPA with GQA, output projection), FeedForward.forward (:268-269), the output head
(:367,394) and the loss of train.py:263-266.
"""
from __future__ import annotations

import math
import os
from typing import Optional, Sequence, Tuple

import torch

from .. import _ext
from . import reference as ref
from . import sched


# ---------------------------------------------------------------------------------------
# gradient slots for modules that are not (yet) flattened
class UnflatSlot:
    """Gradient sink that accumulates into ``p.grad`` for a group of adjacent params."""

    def __init__(self, params: Sequence[torch.nn.Parameter]):
        self.params = list(params)
        self.numel = sum(p.numel() for p in self.params)

    def begin(self, like: torch.Tensor):
        return torch.empty(self.numel, dtype=self.params[0].dtype, device=self.params[0].device), False

    def end(self, buf: torch.Tensor):
        o = 0
        for p in self.params:
            part = buf[o:o + p.numel()].view_as(p)
            if p.grad is None:
                p.grad = part.clone()
            else:
                p.grad.add_(part)
            o += p.numel()

    def mm_(self, a, b, shape):
        buf, _ = self.begin(a)
        torch.mm(a, b, out=buf.view(shape))
        self.end(buf)


class FlatSlotAdapter:
    """begin/end protocol over a :class:`~pyrecover_amd.parallel.flat.GradSlot`."""

    __slots__ = ("s",)

    def __init__(self, s):
        self.s = s

    def begin(self, like):
        return self.s.view, self.s.take()

    def end(self, buf):
        self.s.done()

    def mm_(self, a, b, shape):
        self.s.mm_(a, b, shape)


def _mm_into(slot, a, b, shape):
    slot.mm_(a, b, shape)


# Measured defaults, switchable only from code (tools/step_ab.py arms, tests; no environment knob):
# * TN_WGRAD / TN_WGRAD_WO: library weight gradients dW = dY^T X (K = tokens) run on K-contiguous
#   transposed copies ("TN": dYt [out, T] times Xt [in, T]^T), ~25-30% faster than on the row-major
#   activations, which is worth two bandwidth-bound HIP transposes for the large projections (QKV,
#   output projection, W1|W3, W2, output head; tools/gemm_bench.py --layouts);
# * SWIGLU_BWD_VARIANT: SwiGLU backward kernel (csrc/kernels/elementwise.hip pra_swiglu_bwd), -1 =
#   hoisted tile kernel, 0 = grid-stride kernel;
# * FUSED_ROPE_BWD: inverse RoPE of dq / dk in the attention backward's epilogue (else a separate
#   pass over dq|dk).
SWIGLU_BWD_VARIANT = -1
FUSED_ROPE_BWD = True
TN_WGRAD = True
TN_WGRAD_WO = True


# Shape limits of the HIP kernels (outside them the op runs the torch math of ops/reference.py on
# the same device, like fp64): norms hold a row in registers (D <= 8192, 16-B chunks), embedding
# rows and SwiGLU halves move as 16-B vectors.
_FALLBACK_WARNED = set()


def _note_fallback(op: str, t, ok: bool) -> bool:
    """Warn once per (op, dtype, shape) when a GPU tensor leaves the HIP kernels for the torch
    math of ops/reference.py (an unsupported head_dim, width or dtype): that path is correct
    but can be many times slower (attention materialises the S x S scores)."""
    if not ok and t.is_cuda:
        key = (op, t.dtype, tuple(t.shape[-2:]))
        if key not in _FALLBACK_WARNED:
            _FALLBACK_WARNED.add(key)
            import warnings

            warnings.warn(f"pyrecover_amd: {op} on a {t.dtype} GPU tensor of shape {tuple(t.shape)} runs PyTorch "
                          f"math (outside the HIP kernels' limits)", RuntimeWarning, stacklevel=3)
    return ok


def _norm_hip(x):
    return _note_fallback("norm", x, _ext.hip(x) and x.shape[-1] % 8 == 0 and x.shape[-1] <= 8192)


def _vec_hip(t, width):
    return _note_fallback("elementwise", t, _ext.hip(t) and width % 8 == 0)


def _tn_ok(t):
    return (_ext.hip16(t) and t.dim() == 2 and t.element_size() == 2 and t.stride(1) == 1 and t.size(0) % 64 == 0
            and t.size(1) % 64 == 0 and t.stride(0) % 8 == 0)


# Weight gradients on the hand-written MFMA GEMM (csrc/kernels/gemm_wgrad.hip): dW = dY^T X read
# straight from the row-major activations, transposed inside the LDS read (ds_read_b64_tr_b16), so
# that site needs neither the TN transposes nor a transposing epilogue. On those operands it is
# 13-22% faster than hipBLASLt, but hipBLASLt on K-contiguous copies is faster per GEMM; the kernel
# wins where the library path's copies cost the most (profiles/wgrad_mfma_r2.md).
# PYRECOVER_WGRAD: "auto" (default: the sites where it wins or ties in the step, at >= 16384
# tokens per GEMM: the output projection, whose library path transposes both operands, QKV, whose
# library path needs x^T and the transposing inverse-RoPE epilogue, W1|W3, whose library path needs
# x^T and the transposing SwiGLU-backward epilogue, and the output head, whose dlogits^T copy is
# T x vocab; W2 stays on hipBLASLt TN (-0.5% on the kernel). 7B B16 31.04k vs 30.95k tok/s with
# hipBLASLt TN at every site; Llama-3-8B S8192 B1 (8192 tokens) -0.2%, hence the threshold.
# profiles/wgrad_mfma_r2.md), "hip" (every site), "lib" (none), or a comma list of sites
# (qkv, o, w13, w2, head).
_WGRAD_SITE_SETS = {"lib": frozenset(), "hip": frozenset({"qkv", "o", "w13", "w2", "head"}),
                    "auto": frozenset({"qkv", "o", "w13", "head"})}


def _wgrad_sites(v: str) -> frozenset:
    if v in _WGRAD_SITE_SETS:
        return _WGRAD_SITE_SETS[v]
    sites = frozenset(x.strip() for x in v.split(",") if x.strip())
    bad = sites - _WGRAD_SITE_SETS["hip"]
    if bad:
        raise ValueError(f"PYRECOVER_WGRAD: unknown site(s) {sorted(bad)}")
    return sites


WGRAD_SITES = _wgrad_sites(os.environ.get("PYRECOVER_WGRAD", "auto"))
WGRAD_AUTO = os.environ.get("PYRECOVER_WGRAD", "auto") == "auto"
WGRAD_AUTO_MIN_TOKENS = 16384


def _wgrad_fills_chip(t, cols) -> bool:
    """auto: at least one 256 x 256 output tile per CU. Smaller outputs (GPT-2-medium's 16 / 48 / 88
    tiles) leave most CUs idle on the kernel, which splits only a partial LAST round over K; there
    hipBLASLt's K-split on transposed copies is 1.5-3x faster (profiles/r3/wgrad_bench_gpt2m_*.log:
    QKV 3072x1024x32768 565 vs 321 us, O 574 vs 154 us, W1|W3 596 vs 464 us; step 123.9 -> 103.2 ms)."""
    tiles = 1
    for c in cols:
        tiles *= c // 256
    return tiles >= _cus(t)


def _hip_wgrad_dims(t, site, tokens, *cols, force=False) -> bool:
    """The MFMA weight-gradient kernel's shape rules: K = tokens % 32, every output dim % 256.
    `force`: the operands exist only row-major (no transposed copy to hand the library), so the
    kernel runs whatever the site list and token threshold say (PYRECOVER_WGRAD=lib still wins)."""
    if WGRAD_SITES == _WGRAD_SITE_SETS["lib"] and os.environ.get("PYRECOVER_WGRAD") == "lib":
        force = False
    if not (_ext.hip16(t) and tokens % 32 == 0 and tokens > 0 and all(c % 256 == 0 for c in cols)):
        return False
    return force or (site in WGRAD_SITES and (not WGRAD_AUTO or (tokens >= WGRAD_AUTO_MIN_TOKENS
                                                                 and _wgrad_fills_chip(t, cols))))


def _hip_wgrad_ok(dy2, x2, site, force=False) -> bool:
    return (dy2.dim() == 2 and x2.dim() == 2 and dy2.dtype == x2.dtype and dy2.device == x2.device
            and dy2.size(0) == x2.size(0)
            and _hip_wgrad_dims(dy2, site, dy2.size(0), dy2.size(1), x2.size(1), force=force)
            and all(t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 for t in (dy2, x2)))


def _hip_wgrad(slot, dy2, x2, shape):
    """slot (+)= dy2^T x2 on the MFMA kernel (beta = 1 when the slot already holds a gradient)."""
    if hasattr(slot, "take"):  # flat GradSlot: write into the flat gradient buffer in place
        acc = slot.take()
        _ext.require_for(dy2).wgrad_mm_(dy2, x2, slot.view.view(shape), acc)
        slot.done()
    else:
        buf, acc = slot.begin(dy2)
        _ext.require_for(dy2).wgrad_mm_(dy2, x2, buf.view(shape), acc)
        slot.end(buf)


def _wgrad_into(slot, dy2, x2, shape, site, force=False):
    """slot <- dy2^T x2 (dy2 [T, out], x2 [T, in]); `site` names the projection (WGRAD_SITES)."""
    if _hip_wgrad_ok(dy2, x2, site, force):
        _hip_wgrad(slot, dy2, x2, shape)
    elif TN_WGRAD and _tn_ok(dy2) and _tn_ok(x2):
        C = _ext.require_for(dy2)
        slot.mm_(C.transpose2d(dy2), C.transpose2d(x2).t(), shape)
    else:
        slot.mm_(dy2.t(), x2, shape)


# Forward and data-gradient GEMMs on the hand-written MFMA NT kernel (csrc/kernels/gemm_nt.hip):
# both operands K-contiguous (activations [T, in] x weights [out, in]; the data gradients use the
# transposed weight shadows), with fused epilogues where a separate memory-bound pass followed:
# RoPE on the QKV projection, SwiGLU on the W1|W3 projection, the SwiGLU backward on the W2 data
# gradient. Round 4: the NT kernel runs at 0.90-0.97 of hipBLASLt on the 7B shapes (two-buffer loop,
# M0 writes one MFMA ahead of each LDS-DMA, row offsets in VGPRs, 16-B epilogue stores:
# profiles/r4/gemm_nt_bench_st16.log), and the W1|W3 projection with the SwiGLU epilogue beats
# hipBLASLt + the separate SwiGLU kernel: 4057 vs 4173 us per layer, 7B B16 step 1039.2 -> 1034.9 ms
# (profiles/r4/step_ab_fused_swiglu_st16.log). Plain NT sites stay on hipBLASLt (adding the output
# projection: 1037.4 ms). "auto" therefore runs w13 on the NT kernel. PYRECOVER_GEMM: "auto"
# (default), "hip" (every valid site on the NT kernel), "lib",
# or a comma list of sites: forward qkv, o, w13, w2, head; data gradient qkv_d, o_d, w13_d, w2_d,
# head_d.
_NT_ALL = frozenset({"qkv", "o", "w13", "w2", "head", "qkv_d", "o_d", "w13_d", "w2_d", "head_d"})
_NT_AUTO = frozenset({"w13"})
# ... from this many tokens per GEMM: at 2048 (Llama-3-8B B1 S2048) the fused path, whose W2 weight
# gradient then runs the MFMA kernel on the row-major activation at K = 2048, is 1.8% slower in the
# step; at 8192 (S8192 B1) 0.24% faster (profiles/r4/step_ab_llama3_8b_*_w13.log)
NT_AUTO_MIN_TOKENS = 8192
# ... and from this depth: a 256x256 tile's prologue + SwiGLU epilogue (~24k cycles) is measured
# against a 4096-deep main loop (64 chunks, ~156k cycles); at K = 1024 it is a third of the tile,
# and GPT-2-medium's step runs 6.2% slower with the fused path (104.5 vs 110.9 ms:
# profiles/r4/step_ab_gpt2m_w13_r5l.log, profiles/r4/gemm_nt_swiglu_epilogue_stamps.log)
NT_AUTO_MIN_K = 4096


def _gemm_sites(v: str) -> frozenset:
    if v == "auto":
        return _NT_AUTO
    if v == "hip":
        return _NT_ALL
    if v == "lib":
        return frozenset()
    sites = frozenset(x.strip() for x in v.split(",") if x.strip())
    bad = sites - _NT_ALL
    if bad:
        raise ValueError(f"PYRECOVER_GEMM: unknown site(s) {sorted(bad)}")
    return sites


GEMM_SITES = _gemm_sites(os.environ.get("PYRECOVER_GEMM", "auto"))
GEMM_AUTO = os.environ.get("PYRECOVER_GEMM", "auto") == "auto"
_CUS = {}


def _cus(t) -> int:
    i = t.device.index
    if i not in _CUS:
        _CUS[i] = torch.cuda.get_device_properties(t.device).multi_processor_count
    return _CUS[i]


def _nt_ok(a, b, site) -> bool:
    """out = a b^T on the NT kernel: a [M, K], b [N, K] K-contiguous 16-bit, M, N % 256, K % 32."""
    if site not in GEMM_SITES or b is None or not _ext.hip16(a):
        return False
    if not (a.dim() == 2 and b.dim() == 2 and a.dtype == b.dtype and a.device == b.device
            and a.size(1) == b.size(1) and a.size(0) % 256 == 0 and b.size(0) % 256 == 0 and a.size(1) % 32 == 0):
        return False
    if not all(t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0 for t in (a, b)):
        return False
    return not GEMM_AUTO or ((a.size(0) // 256) * (b.size(0) // 256) >= 2 * _cus(a)
                             and a.size(0) >= NT_AUTO_MIN_TOKENS and a.size(1) >= NT_AUTO_MIN_K)


def _mm_nt(a, b, site, b_t=None):
    """a @ b^T. `b_t` (optional) is b^T stored K-contiguous the other way round: when the NT
    kernel cannot run, the library GEMM uses whichever layout it has."""
    if _nt_ok(a, b, site):
        out = torch.empty(a.size(0), b.size(0), dtype=a.dtype, device=a.device)
        _ext.require_for(a).gemm_nt_(a, b, out)
        return out
    return torch.mm(a, b_t) if b_t is not None else torch.mm(a, b.t())


def _mm_dgrad(dy, w, w_t, site):
    """dX = dY W (w [out, in]); w_t = W^T [in, out] is the K-contiguous shadow the NT kernel reads."""
    if w_t is not None:
        return _mm_nt(dy, w_t, site)
    return torch.mm(dy, w)


# ---------------------------------------------------------------------------------------
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, weight, slot):
        ctx.slot = slot
        ctx.save_for_backward(ids)
        ctx.shape = weight.shape
        if _vec_hip(weight, weight.shape[1]):
            return _ext.require_for(weight).embedding_fwd(ids.contiguous(), weight)
        return torch.nn.functional.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dout):
        (ids,) = ctx.saved_tensors
        slot = ctx.slot
        buf, acc = slot.begin(dout)
        V, D = ctx.shape
        gs = getattr(slot, "s", None)
        if gs is not None:  # the rows this gradient touches, for a sparse exchange (parallel/ddp.py)
            prev = gs.sparse_ids if acc else None
            gs.sparse_ids = ids.reshape(-1) if prev is None else torch.cat([prev, ids.reshape(-1)])
        if _vec_hip(dout, D):
            _ext.require_for(dout).embedding_bwd(ids.contiguous(), dout.contiguous(), buf.view(V, D), acc)
        else:
            g = buf.view(V, D)
            if not acc:
                g.zero_()
            g.index_add_(0, ids.reshape(-1), dout.reshape(-1, D).to(g.dtype))
        slot.end(buf)
        return None, None, None


def embedding(ids, weight, slot):
    return _Embedding.apply(ids, weight, slot)


# ---------------------------------------------------------------------------------------
class _AddRMSNorm(torch.autograd.Function):
    """(h, y) = (x + delta, rmsnorm(x + delta) * w); delta may be None (then h is x)."""

    @staticmethod
    def forward(ctx, x, delta, weight, slot, eps):
        ctx.slot = slot
        ctx.has_delta = delta is not None
        if _norm_hip(x):
            h, y, rstd = _ext.require_for(x).rmsnorm_fwd(x.contiguous(), delta.contiguous() if delta is not None else None,
                                                         weight, eps)
        else:
            h, y, rstd = ref.rmsnorm_fwd(x, delta, weight, eps)
        ctx.save_for_backward(h, weight, rstd)
        if delta is None:
            return y
        return h, y

    @staticmethod
    def backward(ctx, *grads):
        h, weight, rstd = ctx.saved_tensors
        if ctx.has_delta:
            dh, dy = grads
        else:
            dh, dy = None, grads[0]
        slot = ctx.slot
        buf, acc = slot.begin(dy)
        if _norm_hip(dy):
            dx = _ext.require_for(dy).rmsnorm_bwd(dy.contiguous(), h, weight, rstd,
                                                  dh.contiguous() if dh is not None else None, buf, acc)
        else:
            dx, dw = ref.rmsnorm_bwd(dy, h, weight, rstd, dh)
            if acc:
                buf.add_(dw.to(buf.dtype))
            else:
                buf.copy_(dw)
        slot.end(buf)
        if ctx.has_delta:
            return dx, dx, None, None, None
        return dx, None, None, None, None


def add_rms_norm(x, delta, weight, slot, eps):
    """Returns (h, normed) when delta is given, else normed."""
    return _AddRMSNorm.apply(x, delta, weight, slot, eps)


# ---------------------------------------------------------------------------------------
class _AddLayerNorm(torch.autograd.Function):
    """LayerNorm variant (norm_type="layernorm"): (h, y) = (x + delta, layer_norm(x + delta)*w + b).
    Gradients of weight|bias land in one slot (the two params are adjacent in the flat buffer)."""

    @staticmethod
    def forward(ctx, x, delta, weight, bias, slot, eps):
        ctx.slot = slot
        ctx.has_delta = delta is not None
        ctx.eps = eps
        if _norm_hip(x):
            h, y, mean, rstd = _ext.require_for(x).layernorm_fwd(
                x.contiguous(), delta.contiguous() if delta is not None else None, weight, bias, eps)
        else:
            h = x if delta is None else x + delta
            y = torch.nn.functional.layer_norm(h, (h.shape[-1],), weight, bias, eps)
            mean = rstd = torch.empty(0)
        ctx.save_for_backward(h, weight, bias, mean, rstd)
        if delta is None:
            return y
        return h, y

    @staticmethod
    def backward(ctx, *grads):
        h, weight, bias, mean, rstd = ctx.saved_tensors
        dh, dy = grads if ctx.has_delta else (None, grads[0])
        slot = ctx.slot
        buf, acc = slot.begin(dy)
        D = h.shape[-1]
        if _norm_hip(dy):
            dx = _ext.require_for(dy).layernorm_bwd(dy.contiguous(), h, weight, mean, rstd,
                                                    dh.contiguous() if dh is not None else None, buf, acc)
        else:
            with torch.enable_grad():
                hh = h.detach().requires_grad_()
                ww = weight.detach().requires_grad_()
                bb = bias.detach().requires_grad_()
                yy = torch.nn.functional.layer_norm(hh, (D,), ww, bb, ctx.eps)
                gx, gw, gb = torch.autograd.grad(yy, (hh, ww, bb), dy)
            dx = gx if dh is None else gx + dh
            g = torch.cat([gw.reshape(-1), gb.reshape(-1)]).to(buf.dtype)
            if acc:
                buf.add_(g)
            else:
                buf.copy_(g)
        slot.end(buf)
        if ctx.has_delta:
            return dx, dx, None, None, None, None
        return dx, None, None, None, None, None


def add_layer_norm(x, delta, weight, bias, slot, eps):
    return _AddLayerNorm.apply(x, delta, weight, bias, slot, eps)


# ---------------------------------------------------------------------------------------
def _attn_hip(q, k):
    """The MFMA kernels: bf16/fp16 (attention.hip) or fp32 (attention_f32.hip, f32-input MFMA),
    head_dim 64 or 128, whole GQA groups, 16-B aligned rows."""
    return _note_fallback("attention", q, _ext.hip(q) and q.shape[-1] in (64, 128) and q.shape[2] % k.shape[2] == 0
                          and all(t.stride(-1) == 1 and t.stride(1) % 8 == 0 for t in (q, k)))


def _attn_fwd(q, k, v, scale, causal):
    """HIP flash attention for bf16/fp16/fp32 GPU tensors with head_dim 64/128 (any S: the binding
    zero-pads sequences that do not tile); otherwise (fp64, other head dims) torch math in the
    input's precision, as the reference's non-flash path (reference model.py:192, 227).
    Returns (o, lse or None)."""
    if _attn_hip(q, k):
        return _ext.require_for(q).attn_fwd(q, k, v, scale, causal)
    ct = torch.promote_types(q.dtype, torch.float32)
    with torch.no_grad():
        o = ref.attention_ref(q.to(ct), k.to(ct), v.to(ct), causal, scale)
    return o.to(q.dtype).contiguous(), None


def _attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal, rope_tab=None) -> bool:
    """Attention backward into dq/dk/dv. With ``rope_tab`` (the forward's RoPE table) the HIP kernels
    store dq and dk with the inverse rotation already applied; returns whether that happened (the
    torch path leaves it to the caller)."""
    if lse is not None and _attn_hip(q, k):
        if q.dtype == torch.float32:
            rope_tab = None  # the fp32 kernels have no fused inverse RoPE: the caller applies it
        ev = None
        if sched.has_hooks():  # a side-stream job waits for the dK/dV kernel (ops/sched.py)
            ev = torch.cuda.Event()
            ev.record()  # creates the event; the launcher re-records it between dQ and dK/dV
        _ext.require_for(q).attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, causal, rope_tab,
                                     ev.cuda_event if ev is not None else 0)
        if ev is not None:
            sched.attention_window(ev, q.device.index)
        return rope_tab is not None
    ct = torch.promote_types(q.dtype, torch.float32)
    with torch.enable_grad():
        qq, kk, vv = (t.detach().to(ct).requires_grad_() for t in (q, k, v))
        out = ref.attention_ref(qq, kk, vv, causal, scale)
        gq, gk, gv = torch.autograd.grad(out, (qq, kk, vv), do.to(ct))
    dq.copy_(gq)
    dk.copy_(gk)
    dv.copy_(gv)
    return False


class _AttentionBlock(torch.autograd.Function):
    """y = Wo · attn(rope(Wq x), rope(Wk x), Wv x) with a fused QKV GEMM."""

    @staticmethod
    def forward(ctx, x, w_qkv, w_o, slot_qkv, slot_o, tab, dims, w_t, *params):
        B, S, Hq, Hkv, D, causal = dims
        ctx.w_t = w_t  # transposed weight shadows (or None): faster data-gradient GEMM layout
        T = B * S
        dim = x.shape[-1]
        x2 = x.reshape(T, dim)
        nq, nk = Hq * D, Hkv * D
        if _nt_ok(x2, w_qkv, "qkv") and D % 8 == 0 and T % S == 0 and tab.is_contiguous():
            # QKV projection with RoPE on q and k in the GEMM epilogue
            qkv = torch.empty(T, w_qkv.size(0), dtype=x2.dtype, device=x2.device)
            _ext.require_for(x2).gemm_nt_(x2, w_qkv, qkv, 3, None, tab, S, D, nq + nk)
        else:
            qkv = torch.mm(x2, w_qkv.t())
            if _ext.hip(qkv) and D % 8 == 0:
                _ext.require_for(qkv).rope_(qkv, nq + nk, tab, D, S, 0, False)
            else:
                ref.rope_inplace_2d(qkv, nq + nk, tab, D, S)
        q = qkv[:, :nq].view(B, S, Hq, D)
        k = qkv[:, nq:nq + nk].view(B, S, Hkv, D)
        v = qkv[:, nq + nk:].view(B, S, Hkv, D)
        scale = 1.0 / math.sqrt(D)
        o, lse = _attn_fwd(q, k, v, scale, causal)
        o2 = o.view(T, nq)
        y = _mm_nt(o2, w_o, "o")
        ctx.save_for_backward(x2, qkv, o, lse, w_qkv, w_o, tab)
        ctx.slots = (slot_qkv, slot_o)
        ctx.dims = dims
        ctx.scale = scale
        return y.view(B, S, dim)

    @staticmethod
    def backward(ctx, dy):
        x2, qkv, o, lse, w_qkv, w_o, tab = ctx.saved_tensors
        slot_qkv, slot_o = ctx.slots
        B, S, Hq, Hkv, D, causal = ctx.dims
        T = B * S
        nq, nk = Hq * D, Hkv * D
        dy2 = dy.reshape(T, -1)
        o2 = o.view(T, nq)
        # every read of a weight is enqueued BEFORE its gradient slot is published: a published
        # slot may be updated by the optimizer (overlapped with backward) on another stream.
        w_qkv_t, w_o_t = ctx.w_t if ctx.w_t is not None else (None, None)
        do = _mm_dgrad(dy2, w_o, w_o_t, "o_d").view(B, S, Hq, D)
        if TN_WGRAD_WO:
            _wgrad_into(slot_o, dy2, o2, tuple(w_o.shape), "o")
        else:
            slot_o.mm_(dy2.t(), o2, tuple(w_o.shape))
        dqkv = torch.empty_like(qkv)
        q = qkv[:, :nq].view(B, S, Hq, D)
        k = qkv[:, nq:nq + nk].view(B, S, Hkv, D)
        v = qkv[:, nq + nk:].view(B, S, Hkv, D)
        dq = dqkv[:, :nq].view(B, S, Hq, D)
        dk = dqkv[:, nq:nq + nk].view(B, S, Hkv, D)
        dv = dqkv[:, nq + nk:].view(B, S, Hkv, D)
        # the HIP backward applies the inverse RoPE to dq / dk in its epilogue (table rows = positions)
        use_tab = FUSED_ROPE_BWD and tab.is_contiguous() and tab.dtype == torch.float32 and tab.shape[0] >= S
        fused_rope = _attn_bwd(q, k, v, o, do, lse, dq, dk, dv, ctx.scale, causal, tab if use_tab else None)
        if (not _hip_wgrad_ok(dqkv, x2, "qkv") and TN_WGRAD and _tn_ok(dqkv) and _tn_ok(x2) and T % S == 0
                and D % 8 == 0):
            # (inverse RoPE in place +) dqkv^T in one pass, for the K-contiguous weight-grad GEMM
            C = _ext.require_for(dqkv)
            dqkvT = C.transpose2d(dqkv) if fused_rope else C.rope_t_(dqkv, nq + nk, tab, D, S, True)
            dx = _mm_dgrad(dqkv, w_qkv, w_qkv_t, "qkv_d")
            slot_qkv.mm_(dqkvT, C.transpose2d(x2).t(), tuple(w_qkv.shape))
        else:
            if fused_rope:
                pass  # dq / dk already un-rotated by the attention backward
            elif _ext.hip(dqkv) and D % 8 == 0:
                _ext.require_for(dqkv).rope_(dqkv, nq + nk, tab, D, S, 0, True)
            else:
                ref.rope_inplace_2d(dqkv, nq + nk, tab, D, S, inverse=True)
            dx = _mm_dgrad(dqkv, w_qkv, w_qkv_t, "qkv_d")
            _wgrad_into(slot_qkv, dqkv, x2, tuple(w_qkv.shape), "qkv")
        n_params = ctx.needs_input_grad.__len__() - 8
        return (dx.view(B, S, -1), None, None, None, None, None, None, None) + (None,) * n_params


def attention_block(x, w_qkv, w_o, slot_qkv, slot_o, tab, dims, params, w_t=None):
    if w_t is not None and any(t is None for t in w_t):
        w_t = None
    return _AttentionBlock.apply(x, w_qkv, w_o, slot_qkv, slot_o, tab, dims, w_t, *params)


# ---------------------------------------------------------------------------------------
def _swiglu_fwd(gu):
    if _vec_hip(gu, gu.shape[1] // 2) and gu.shape[1] % 16 == 0:
        return _ext.require_for(gu).swiglu_fwd(gu)
    F = gu.shape[1] // 2
    g, u = ref.up(gu[:, :F]), ref.up(gu[:, F:])
    return (ref.up(torch.nn.functional.silu(g).to(gu.dtype)) * u).to(gu.dtype)


def _swiglu_bwd_(da, gu):
    if _vec_hip(gu, gu.shape[1] // 2) and gu.shape[1] % 16 == 0:
        return _ext.require_for(gu).swiglu_bwd(da, gu, gu, SWIGLU_BWD_VARIANT)
    F = gu.shape[1] // 2
    dg, du = ref.swiglu_bwd_ref(da, gu[:, :F], gu[:, F:])
    gu[:, :F] = dg
    gu[:, F:] = du
    return gu


class _SwiGLUMLP(torch.autograd.Function):
    """y = W2 (silu(W1 x) * (W3 x)) with W1|W3 fused into one GEMM."""

    @staticmethod
    def forward(ctx, x, w13, w2, slot13, slot2, w_t, *params):
        ctx.w_t = w_t
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        F = w13.shape[0] // 2
        ctx.fused_act = False
        if _nt_ok(x2, w13, "w13") and F % 128 == 0:
            # W1|W3 projection with the SwiGLU epilogue: writes gu (kept for the backward) and a
            gu = torch.empty(x2.size(0), 2 * F, dtype=x2.dtype, device=x2.device)
            a = a_saved = torch.empty(x2.size(0), F, dtype=x2.dtype, device=x2.device)
            _ext.require_for(x2).gemm_nt_(x2, w13, gu, 1, a)
            ctx.a_is_t = False
            ctx.fused_act = True
        else:
            gu = torch.mm(x2, w13.t())
            if (not _hip_wgrad_dims(gu, "w2", gu.shape[0], shape[-1], F) and TN_WGRAD and _tn_ok(gu)
                    and F % 64 == 0):
                # a^T (K-contiguous operand of the W2 weight gradient) is written in the same pass
                # and kept instead of a
                a, a_saved = _ext.require_for(gu).swiglu_fwd_t(gu)
                ctx.a_is_t = True
            else:
                a = a_saved = _swiglu_fwd(gu)
                ctx.a_is_t = False
        y = _mm_nt(a, w2, "w2")
        ctx.save_for_backward(x2, gu, a_saved, w13, w2)
        ctx.slots = (slot13, slot2)
        return y.view(shape)

    @staticmethod
    def _w2_wgrad(ctx, slot2, dy2, a, w2):
        if ctx.a_is_t:  # TN weight gradient: dW2 = (dY^T) (a^T)^T, both operands K-contiguous
            dyT = _ext.require_for(dy2).transpose2d(dy2) if _tn_ok(dy2) else dy2.t()
            slot2.mm_(dyT, a.t(), tuple(w2.shape))
        else:  # a exists only row-major after the fused SwiGLU epilogue: the MFMA kernel reads it as is
            _wgrad_into(slot2, dy2, a, tuple(w2.shape), "w2", force=ctx.fused_act)

    @staticmethod
    def backward(ctx, dy):
        x2, gu, a, w13, w2 = ctx.saved_tensors
        slot13, slot2 = ctx.slots
        shape = dy.shape
        dy2 = dy.reshape(-1, shape[-1])
        w13_t, w2_t = ctx.w_t if ctx.w_t is not None else (None, None)
        F = gu.shape[1] // 2
        if _nt_ok(dy2, w2_t, "w2_d") and F % 256 == 0:
            # W2 data gradient with the SwiGLU backward in the epilogue: da never leaves the
            # registers; g, u in gu are overwritten with dg, du
            _ext.require_for(dy2).gemm_nt_(dy2, w2_t, gu, 2)
            _SwiGLUMLP._w2_wgrad(ctx, slot2, dy2, a, w2)
            dgu = gu
            dx = _mm_dgrad(dgu, w13, w13_t, "w13_d")
            _wgrad_into(slot13, dgu, x2, tuple(w13.shape), "w13", force=True)
            n_params = len(ctx.needs_input_grad) - 6
            return (dx.view(shape), None, None, None, None, None) + (None,) * n_params
        da = _mm_dgrad(dy2, w2, w2_t, "w2_d")
        _SwiGLUMLP._w2_wgrad(ctx, slot2, dy2, a, w2)
        if _hip_wgrad_ok(gu, x2, "w13"):
            dgu = _swiglu_bwd_(da, gu)  # in place over gu; no transposed copy for the MFMA wgrad
            dx = _mm_dgrad(dgu, w13, w13_t, "w13_d")
            _hip_wgrad(slot13, dgu, x2, tuple(w13.shape))
        elif TN_WGRAD and _tn_ok(gu) and _tn_ok(x2) and _tn_ok(da):
            # SwiGLU backward in place over gu, writing dgu^T in the same pass
            C = _ext.require_for(gu)
            dguT = C.swiglu_bwd_t_(da, gu)
            dx = _mm_dgrad(gu, w13, w13_t, "w13_d")
            slot13.mm_(dguT, C.transpose2d(x2).t(), tuple(w13.shape))
        else:
            dgu = _swiglu_bwd_(da, gu)  # in place over gu (dead after this)
            dx = _mm_dgrad(dgu, w13, w13_t, "w13_d")
            _wgrad_into(slot13, dgu, x2, tuple(w13.shape), "w13")
        n_params = len(ctx.needs_input_grad) - 6
        return (dx.view(shape), None, None, None, None, None) + (None,) * n_params


def swiglu_mlp(x, w13, w2, slot13, slot2, params, w_t=None):
    if w_t is not None and any(t is None for t in w_t):
        w_t = None
    return _SwiGLUMLP.apply(x, w13, w2, slot13, slot2, w_t, *params)


# ---------------------------------------------------------------------------------------
class _LinearCrossEntropy(torch.autograd.Function):
    """loss = CE(h · Wout^T, labels, sum) / #valid; logits never leave bf16 and are turned into
    dlogits in place during the backward."""

    @staticmethod
    def forward(ctx, h, w_out, labels, slot, ignore_index, w_t, weight_param):
        ctx.w_t = w_t
        h2 = h.reshape(-1, h.shape[-1])
        lab = labels.reshape(-1).contiguous()
        logits = _mm_nt(h2, w_out, "head")
        if _ext.hip(logits):
            lse, _, stats = _ext.require_for(logits).xent_fwd(logits, lab, ignore_index)
            loss = stats[0]
        else:
            lse = torch.logsumexp(ref.up(logits), dim=-1)
            stats = None
            loss = ref.cross_entropy_ref(logits, lab, ignore_index)
        ctx.save_for_backward(h2, logits, lab, lse, w_out, stats if stats is not None else lse)
        ctx.slot = slot
        ctx.ignore_index = ignore_index
        ctx.hshape = h.shape
        return loss

    @staticmethod
    def backward(ctx, dloss):
        h2, logits, lab, lse, w_out, stats = ctx.saved_tensors
        if _ext.hip(logits):
            g = dloss.reshape(1).float().contiguous()
            _ext.require_for(logits).xent_bwd_(logits, lab, lse, stats, g, ctx.ignore_index)
            dlogits = logits
        else:
            valid = lab.ne(ctx.ignore_index)
            n = valid.sum().clamp_min(1)
            p = torch.softmax(ref.up(logits), dim=-1)
            p[torch.arange(lab.numel(), device=p.device), lab.clamp_min(0)] -= valid.to(p.dtype)
            p = p * valid.to(p.dtype).unsqueeze(1) * (dloss.to(p.dtype) / n)
            dlogits = p.to(logits.dtype)
        dh = _mm_dgrad(dlogits, w_out, ctx.w_t, "head_d")
        _wgrad_into(ctx.slot, dlogits, h2, tuple(w_out.shape), "head")
        return dh.view(ctx.hshape), None, None, None, None, None, None


def linear_cross_entropy(h, w_out, labels, slot, weight_param, ignore_index: int = -100, w_t=None):
    return _LinearCrossEntropy.apply(h, w_out, labels, slot, ignore_index, w_t, weight_param)


# ---------------------------------------------------------------------------------------
# Standalone user-facing ops (autograd, no slots)
class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = _attn_fwd(q, k, v, scale, causal)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _attn_bwd(q, k, v, o, do.contiguous(), lse, dq, dk, dv, ctx.scale, ctx.causal)
        return dq, dk, dv, None, None


def flash_attention(q, k, v, causal: bool = True, scale: Optional[float] = None):
    """Causal/full GQA attention on [B, S, H, D] tensors (HIP MFMA kernel on GPU)."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    return _FlashAttention.apply(q, k, v, causal, scale)
