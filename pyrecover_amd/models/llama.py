"""Llama-style decoder with the reference's parameter names, shapes, order and init.

Module tree and state-dict keys are identical to reference model.py:330-395
(``tok_embeddings``, ``layers.{i}.attention.{wq,wk,wv,wo}``, ``layers.{i}.feed_forward.{w1,w2,w3}``,
``layers.{i}.{attention_norm,ffn_norm}``, ``norm``, ``output``; ``freqs_cis`` is a non-persistent
buffer), and parameters are created in the same order with the same ``nn.Linear`` /
``nn.Embedding`` initializers, so a seeded CPU construction is bit-identical to the reference's.

The forward is NOT the reference's module-by-module composition: it runs the fused ops of
:mod:`pyrecover_amd.ops` (fused residual-add + RMSNorm, fused QKV GEMM + in-place RoPE + HIP flash
attention with native GQA, fused W1|W3 GEMM + SwiGLU, fused output GEMM + cross-entropy), and
after :meth:`Transformer.flatten_` all parameters/gradients live in flat buffers
(:mod:`pyrecover_amd.parallel.flat`).
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.utils.checkpoint

from ..config import TransformerModelArgs
from ..ops import fused as F
from ..ops.reference import precompute_freqs_cis, rope_table
from ..parallel.flat import FlatParams


class RMSNorm(nn.Module):
    """Parameter container + reference-compatible eager forward (reference model.py:25-49)."""

    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).type_as(x) * self.weight


class LayerNorm(nn.Module):
    """norm_type="layernorm" (the reference's TransformerModelArgs.norm_type field, model.py:18)."""

    def __init__(self, dim: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim))
        self.bias = nn.Parameter(torch.zeros(dim))

    def forward(self, x):
        return torch.nn.functional.layer_norm(x, (x.shape[-1],), self.weight, self.bias, self.eps)


def make_norm(args: TransformerModelArgs, dim: int):
    if args.norm_type == "rmsnorm":
        return RMSNorm(dim, eps=args.norm_eps)
    if args.norm_type == "layernorm":
        return LayerNorm(dim, eps=args.norm_eps)
    raise ValueError(f"unknown norm_type {args.norm_type!r}")


class Attention(nn.Module):
    def __init__(self, args: TransformerModelArgs):
        super().__init__()
        self.n_heads = args.n_heads
        self.n_kv_heads = args.kv_heads
        self.n_rep = self.n_heads // self.n_kv_heads
        self.head_dim = args.dim // args.n_heads
        self.wq = nn.Linear(args.dim, args.n_heads * self.head_dim, bias=False)
        self.wk = nn.Linear(args.dim, self.n_kv_heads * self.head_dim, bias=False)
        self.wv = nn.Linear(args.dim, self.n_kv_heads * self.head_dim, bias=False)
        self.wo = nn.Linear(args.n_heads * self.head_dim, args.dim, bias=False)
        self.use_flash_attention = args.use_flash_attention  # accepted for CLI parity; HIP flash always used on GPU

    def forward(self, x: torch.Tensor, freqs_cis: torch.Tensor) -> torch.Tensor:
        """Standalone module forward with the reference signature (reference model.py:194-230):
        QKV projections, RoPE from ``freqs_cis`` (complex [>=S, head_dim/2]), causal GQA
        attention, output projection. Runs the same fused op as :class:`Transformer` (one QKV
        GEMM, in-place RoPE, HIP flash attention); weight gradients accumulate into ``.grad``."""
        B, S, _ = x.shape
        qkv = [self.wq.weight, self.wk.weight, self.wv.weight]
        tab = rope_table(freqs_cis[:S].to(x.device))
        dims = (B, S, self.n_heads, self.n_kv_heads, self.head_dim, True)
        return F.attention_block(x, torch.cat([w.detach() for w in qkv], 0), self.wo.weight.detach(),
                                 F.UnflatSlot(qkv), F.UnflatSlot([self.wo.weight]), tab, dims,
                                 qkv + [self.wo.weight])


class FeedForward(nn.Module):
    def __init__(self, dim: int, hidden_dim: int, multiple_of: int, ffn_dim_multiplier: Optional[float]):
        super().__init__()
        hidden_dim = int(2 * hidden_dim / 3)
        if ffn_dim_multiplier is not None:
            hidden_dim = int(ffn_dim_multiplier * hidden_dim)
        hidden_dim = multiple_of * ((hidden_dim + multiple_of - 1) // multiple_of)
        self.w1 = nn.Linear(dim, hidden_dim, bias=False)
        self.w2 = nn.Linear(hidden_dim, dim, bias=False)
        self.w3 = nn.Linear(dim, hidden_dim, bias=False)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        """w2(silu(w1 x) * w3 x) (reference model.py:268-269) as the fused W1|W3 GEMM + SwiGLU op."""
        up = [self.w1.weight, self.w3.weight]
        return F.swiglu_mlp(x, torch.cat([w.detach() for w in up], 0), self.w2.weight.detach(),
                            F.UnflatSlot(up), F.UnflatSlot([self.w2.weight]), up + [self.w2.weight])


class TransformerBlock(nn.Module):
    def __init__(self, layer_id: int, args: TransformerModelArgs):
        super().__init__()
        self.n_heads = args.n_heads
        self.dim = args.dim
        self.attention = Attention(args)
        self.feed_forward = FeedForward(args.dim, 4 * args.dim, args.multiple_of, args.ffn_dim_multiplier)
        self.layer_id = layer_id
        self.num_layers = args.n_layers
        self.attention_norm = make_norm(args, args.dim)
        self.ffn_norm = make_norm(args, args.dim)

    def _norm(self, mod, x, delta):
        if isinstance(mod, LayerNorm):
            return F.add_layer_norm(x, delta, mod.weight, mod.bias, F.UnflatSlot([mod.weight, mod.bias]), mod.eps)
        return F.add_rms_norm(x, delta, mod.weight, F.UnflatSlot([mod.weight]), mod.eps)

    def forward(self, x: torch.Tensor, freqs_cis: torch.Tensor) -> torch.Tensor:
        """h = x + attention(attention_norm(x)); out = h + feed_forward(ffn_norm(h))
        (reference model.py:325-327); the first residual add is fused into ffn_norm."""
        h, n2 = self._norm(self.ffn_norm, x, self.attention(self._norm(self.attention_norm, x, None), freqs_cis))
        return h + self.feed_forward(n2)


class Transformer(nn.Module):
    def __init__(self, model_args: TransformerModelArgs):
        super().__init__()
        if model_args.vocab_size <= 0:
            raise ValueError("vocab_size must be set")
        self.model_args = model_args
        self.vocab_size = model_args.vocab_size
        self.n_layers = model_args.n_layers
        self.tok_embeddings = nn.Embedding(model_args.vocab_size, model_args.dim)
        dev = self.tok_embeddings.weight.device  # honour a `with torch.device(...)` construction
        self.register_buffer("freqs_cis", self._precompute_freqs_cis().to(dev), persistent=False)
        self.layers = nn.ModuleDict()
        for layer_id in range(model_args.n_layers):
            self.layers[str(layer_id)] = TransformerBlock(layer_id, model_args)
        self.norm = make_norm(model_args, model_args.dim)
        self.output = nn.Linear(model_args.dim, model_args.vocab_size, bias=False)
        self.register_buffer("rope_tab", rope_table(self.freqs_cis), persistent=False)
        self.flat: Optional[FlatParams] = None
        self.activation_checkpointing = False  # train.py --activation-checkpointing

    def _precompute_freqs_cis(self) -> torch.Tensor:
        a = self.model_args
        with torch.device("cpu"):
            fc = precompute_freqs_cis(a.dim // a.n_heads, a.seq_len, a.rope_theta)
        return fc

    def _apply(self, fn, recurse=True):
        # the rotation tables never take the model's dtype: keep them out of `fn` (a complex
        # buffer cast to a real dtype would lose its imaginary part) and only follow the device
        tables = {k: self._buffers.pop(k) for k in ("freqs_cis", "rope_tab")}
        try:
            out = super()._apply(fn, recurse)
        finally:
            dev = self.tok_embeddings.weight.device
            for k, t in tables.items():
                self._buffers[k] = t.to(dev)
        if self.flat is not None and any(p.data.data_ptr() < self.flat.data.data_ptr() or
                                         p.data.data_ptr() >= self.flat.data.data_ptr() + self.flat.state_bytes()
                                         for p in self.parameters()):
            self.flat = None  # a .to()/.half() replaced the storages: flat views are gone
        return out

    # ----------------------------------------------------------------------------------
    def fusion_groups(self) -> List[List[Tuple[str, nn.Parameter]]]:
        """Flat-buffer layout in forward order (gradients become ready in reverse order, so DDP
        buckets are contiguous tail-first slices). Adjacent members form fused GEMM weights."""
        def norm_group(prefix, mod):
            grp = [(prefix + "weight", mod.weight)]
            if getattr(mod, "bias", None) is not None:
                grp.append((prefix + "bias", mod.bias))
            return grp

        g = [[("tok_embeddings.weight", self.tok_embeddings.weight)]]
        for i, layer in self.layers.items():
            p = f"layers.{i}."
            at, ff = layer.attention, layer.feed_forward
            g.append(norm_group(p + "attention_norm.", layer.attention_norm))
            g.append([(p + "attention.wq.weight", at.wq.weight), (p + "attention.wk.weight", at.wk.weight),
                      (p + "attention.wv.weight", at.wv.weight)])
            g.append([(p + "attention.wo.weight", at.wo.weight)])
            g.append(norm_group(p + "ffn_norm.", layer.ffn_norm))
            g.append([(p + "feed_forward.w1.weight", ff.w1.weight), (p + "feed_forward.w3.weight", ff.w3.weight)])
            g.append([(p + "feed_forward.w2.weight", ff.w2.weight)])
        g.append(norm_group("norm.", self.norm))
        g.append([("output.weight", self.output.weight)])
        return g

    SHADOW_SITES = ("qkv", "o", "w13", "w2", "head")

    def flatten_(self, tokens_per_step: Optional[int] = None, shadows=None) -> FlatParams:
        """Move all parameters/gradients into flat buffers (call after the final .to(device/dtype)).

        Transposed weight shadows (K-contiguous W^T for the data-gradient GEMMs, rewritten by the
        optimizer), measured with bench.py on MI355X (profiles/r6/shadows/): +3.5% at 7B B16, +7.6% at
        7B B1, +1.3% at 7B B4, +2% at Llama-3-8B S8192 B1, but -1.5% at Llama-3-8B S2048 B1, where no
        single site accounts for it (dropping any one of qkv / o / w13 / w2 / head moves the step by
        -0.4..+0.4%; dropping all of them, the optimizer runs the plain flat update instead of the
        transposing one). ``shadows`` (default: env PRA_WEIGHT_SHADOWS, "auto") is "auto" (every
        site, except none for a grouped-query model at <= 4096 tokens per step), True / "1" (every
        site), False / "0" (none: e.g. the sharded optimizer, whose owned chunks cut matrices and
        would re-derive every shadow after the parameter all-gather) or a comma list of
        SHADOW_SITES.
        """
        if self.flat is None:
            self.flat = FlatParams(self.fusion_groups())
            # optimizer-state indices follow model.parameters() order, as in the reference
            self.flat.module_order = list(self.parameters())
            self.flat.shadow_sites = self.planned_shadow_sites(tokens_per_step, shadows)
            for mats in self._gemm_weights(self.flat.shadow_sites):
                self.flat.register_transposed(mats, (sum(p.shape[0] for p in mats), mats[0].shape[1]))
            # parameters written through the module API must refresh the transposed shadows
            self.register_load_state_dict_post_hook(lambda mod, keys: mod.flat.refresh_transposed())
        return self.flat

    def planned_shadow_sites(self, tokens_per_step: Optional[int] = None, shadows=None) -> Tuple[str, ...]:
        """The sites flatten_ gives a shadow (before any buffer exists; the shadows themselves are only
        registered for 16-bit GPU buffers)."""
        if shadows is None:
            shadows = os.environ.get("PRA_WEIGHT_SHADOWS", "auto")
        if str(shadows).strip().lower() == "auto":
            gqa = self.model_args.kv_heads < self.model_args.n_heads
            shadows = not (gqa and tokens_per_step is not None and tokens_per_step <= 4096)
        return self.shadow_sites(shadows)

    @classmethod
    def shadow_sites(cls, spec) -> Tuple[str, ...]:
        if spec is True or str(spec).strip().lower() in ("1", "all", "true"):
            return cls.SHADOW_SITES
        if spec is False or str(spec).strip().lower() in ("0", "none", "false", ""):
            return ()
        sites = tuple(s.strip() for s in str(spec).split(",") if s.strip())
        bad = [s for s in sites if s not in cls.SHADOW_SITES]
        if bad:
            raise ValueError(f"unknown weight-shadow sites {bad}; choose from {cls.SHADOW_SITES}")
        return sites

    def _gemm_weights(self, sites: Sequence[str] = SHADOW_SITES) -> List[List[nn.Parameter]]:
        out = []
        for layer in self.layers.values():
            at, ff = layer.attention, layer.feed_forward
            per = {"qkv": [at.wq.weight, at.wk.weight, at.wv.weight], "o": [at.wo.weight],
                   "w13": [ff.w1.weight, ff.w3.weight], "w2": [ff.w2.weight]}
            out += [per[s] for s in ("qkv", "o", "w13", "w2") if s in sites]
        if "head" in sites:
            out.append([self.output.weight])
        return out

    def _weight_t(self, params: Sequence[nn.Parameter]) -> Optional[torch.Tensor]:
        return self.flat.weight_t(params) if self.flat is not None else None

    # ----------------------------------------------------------------------------------
    def _slot(self, params: Sequence[nn.Parameter]):
        if self.flat is not None:
            return F.FlatSlotAdapter(self.flat.slot(params[0]))
        return F.UnflatSlot(params)

    def _weight(self, params: Sequence[nn.Parameter]) -> torch.Tensor:
        rows = sum(p.shape[0] for p in params)
        if self.flat is not None:
            return self.flat.weight(params, (rows, params[0].shape[1]))
        if len(params) == 1:
            return params[0].detach()
        return torch.cat([p.detach() for p in params], 0)

    def _norm(self, mod, x, delta):
        if isinstance(mod, LayerNorm):
            return F.add_layer_norm(x, delta, mod.weight, mod.bias, self._slot([mod.weight, mod.bias]), mod.eps)
        return F.add_rms_norm(x, delta, mod.weight, self._slot([mod.weight]), mod.eps)

    def _block(self, layer, h, pending, B: int, S: int):
        """One TransformerBlock (reference model.py:325-327): returns (residual stream, the MLP
        output still to be added -- the add is fused into the next norm)."""
        a = self.model_args
        dims = (B, S, a.n_heads, a.kv_heads, a.head_dim, True)
        at, ff = layer.attention, layer.feed_forward
        if pending is None:
            x, n1 = h, self._norm(layer.attention_norm, h, None)
        else:
            x, n1 = self._norm(layer.attention_norm, h, pending)
        qkv_p = [at.wq.weight, at.wk.weight, at.wv.weight]
        att = F.attention_block(n1, self._weight(qkv_p), self._weight([at.wo.weight]), self._slot(qkv_p),
                                self._slot([at.wo.weight]), self.rope_tab, dims, qkv_p + [at.wo.weight],
                                w_t=(self._weight_t(qkv_p), self._weight_t([at.wo.weight])))
        x2, n2 = self._norm(layer.ffn_norm, x, att)
        up = [ff.w1.weight, ff.w3.weight]
        mlp = F.swiglu_mlp(n2, self._weight(up), self._weight([ff.w2.weight]), self._slot(up),
                           self._slot([ff.w2.weight]), up + [ff.w2.weight],
                           w_t=(self._weight_t(up), self._weight_t([ff.w2.weight])))
        return x2, mlp

    def _trunk(self, tokens: torch.Tensor):
        a = self.model_args
        B, S = tokens.shape
        if S > a.seq_len:
            raise ValueError(f"sequence length {S} exceeds model seq_len {a.seq_len}")
        emb = self.tok_embeddings.weight
        h = F.embedding(tokens, emb, self._slot([emb]))
        pending = None
        recompute = self.activation_checkpointing and torch.is_grad_enabled()
        for layer in self.layers.values():
            if recompute:
                # keep only the block's inputs; its forward is re-run right before its backward
                # (its weights are still un-updated then: a gradient bucket completes only after
                # the lowest layer it covers has finished backward)
                h, pending = torch.utils.checkpoint.checkpoint(self._block, layer, h, pending, B, S,
                                                               use_reentrant=False)
            else:
                h, pending = self._block(layer, h, pending, B, S)
        if pending is None:
            return self._norm(self.norm, h, None)
        _, nf = self._norm(self.norm, h, pending)
        return nf

    def forward(self, tokens: torch.Tensor, labels: Optional[torch.Tensor] = None, ignore_index: int = -100):
        """logits (B, S, V) like the reference, or the mean causal-LM loss when labels are given
        (fused output GEMM + cross-entropy, equal to reference train.py:263-266)."""
        nf = self._trunk(tokens)
        W = self.output.weight
        if labels is not None:
            return F.linear_cross_entropy(nf, self._weight([W]), labels, self._slot([W]), W, ignore_index,
                                          w_t=self._weight_t([W]))
        return torch.nn.functional.linear(nf, W)

    # ----------------------------------------------------------------------------------
    def num_params(self, exclude_embedding: bool = False) -> int:
        n = sum(p.numel() for p in self.parameters())
        if exclude_embedding:
            n -= self.tok_embeddings.weight.numel()
        return n
