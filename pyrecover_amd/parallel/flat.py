"""Flat parameter / gradient space.

MI355X-first replacement for the per-tensor parameter handling that the reference gets from
``nn.Module`` + ``DistributedDataParallel`` (reference train.py:107-122): every trainable
parameter lives in ONE contiguous device buffer, every gradient in a second one with the same
layout. Consequences:

* fused GEMMs: adjacent parameters (wq|wk|wv, w1|w3) form one weight matrix view, so QKV and
  the SwiGLU up-projection are single hipBLASLt GEMMs, and their weight gradients are written by
  one GEMM straight into the flat gradient buffer (no AccumulateGrad copy, no grad zeroing pass);
* DDP buckets are contiguous slices of the gradient buffer, all-reduced in place (no bucket
  copy-in/copy-out);
* the optimizer is one streaming kernel over four flat buffers (param/grad/m/v);
* checkpoint snapshots are a handful of large D2H copies.

Parameters keep their identity and names: ``p.data`` and ``p.grad`` are re-pointed to views of
the flat buffers, so ``model.state_dict()`` / ``model.parameters()`` are unchanged.

Gradient write protocol: each fusion group owns a :class:`GradSlot`. ``zero_grad()`` marks all
slots *fresh* (no memory traffic); the first producer of a step overwrites (beta=0 GEMM), later
producers (gradient accumulation) add. Parameters not covered by a fused op get ordinary
autograd accumulation into their (zeroed) view and report readiness through a
post-accumulate-grad hook.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch

ALIGN = 64  # elements; every group starts 128-B aligned for bf16 (16-B vector loads need 8)


class GradSlot:
    __slots__ = ("flat", "index", "params", "offset", "numel", "view", "fresh", "bucket", "fused", "sparse_ids")

    def __init__(self, flat, index, params, offset, numel, fused):
        self.flat = flat
        self.index = index
        self.params = params
        self.offset = offset
        self.numel = numel
        self.view = flat.grad[offset:offset + numel]
        self.fresh = True
        self.bucket = -1
        self.fused = fused
        self.sparse_ids = None  # token ids behind an embedding gradient (sparse exchange, parallel/ddp.py)

    # --- producers ------------------------------------------------------------------
    def mm_(self, a: torch.Tensor, b: torch.Tensor, shape: Tuple[int, int]):
        """grad(slot) (+)= a @ b, written in place into the flat gradient buffer."""
        out = self.view.view(shape)
        if self.fresh:
            torch.mm(a, b, out=out)
            self.fresh = False
        else:
            out.addmm_(a, b)
        self.flat._ready(self)

    def take(self) -> bool:
        """Claim the slot for a custom producer; returns True if it must accumulate."""
        acc = not self.fresh
        self.fresh = False
        return acc

    def done(self):
        self.flat._ready(self)


class FlatParams:
    """Owns the flat parameter + gradient buffers for a list of fusion groups."""

    def __init__(self, groups: Sequence[Sequence[Tuple[str, torch.nn.Parameter]]], fused_flags: Sequence[bool] = None,
                 device=None, dtype=None):
        flat_groups = [list(g) for g in groups if len(g)]
        all_params = [p for g in flat_groups for _, p in g]
        if len({id(p) for p in all_params}) != len(all_params):
            raise ValueError("a parameter appears in more than one fusion group")
        self.device = torch.device(device) if device is not None else all_params[0].device
        self.dtype = dtype if dtype is not None else all_params[0].dtype
        offs, off = [], 0
        for g in flat_groups:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            offs.append(off)
            off += sum(p.numel() for _, p in g)
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN
        self.data = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.slots: List[GradSlot] = []
        self.slot_of: Dict[int, GradSlot] = {}
        self.param_offset: Dict[int, int] = {}
        self.names: Dict[int, str] = {}
        fused_flags = list(fused_flags) if fused_flags is not None else [True] * len(flat_groups)
        with torch.no_grad():
            for gi, (g, goff) in enumerate(zip(flat_groups, offs)):
                o = goff
                for name, p in g:
                    n = p.numel()
                    view = self.data[o:o + n].view_as(p)
                    view.copy_(p.data)
                    p.data = view
                    p.grad = self.grad[o:o + n].view_as(p)
                    self.param_offset[id(p)] = o
                    self.names[id(p)] = name
                    o += n
                slot = GradSlot(self, gi, [p for _, p in g], goff, o - goff, fused_flags[gi])
                self.slots.append(slot)
                for _, p in g:
                    self.slot_of[id(p)] = slot
        self.params = all_params
        self.reducer = None
        self._hooks = []
        for slot in self.slots:
            if not slot.fused:
                for p in slot.params:
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(slot)))
        self._pending_unfused: Dict[int, int] = {}

    # --- layout for the sharded optimizer -------------------------------------------------
    def relayout(self, buckets: Sequence[Sequence[int]], multiple: int) -> List[Tuple[int, int]]:
        """Re-place the fusion groups so every bucket (a list of consecutive slot indices) spans a
        multiple of ``multiple`` elements, zero padding after its last group; returns the buckets'
        new [lo, hi) ranges, indexed like ``buckets``. The sharded reducer uses it so each bucket
        splits into W equal chunks with no remainder: its reduce-scatter then covers the bucket
        exactly as the all-reduce would (same chunking, same summation order). Parameter values
        move with their groups; call before an optimizer is bound to the buffers."""
        if getattr(self, "layout_frozen", False):
            raise RuntimeError("relayout after an optimizer was bound to the flat buffers")
        order = sorted(range(len(buckets)), key=lambda b: min(buckets[b]))
        new_off: Dict[int, int] = {}
        ranges: List[Tuple[int, int]] = [(0, 0)] * len(buckets)
        off = 0
        for b in order:
            start = off = (off + ALIGN - 1) // ALIGN * ALIGN
            for gi in sorted(buckets[b]):
                off = (off + ALIGN - 1) // ALIGN * ALIGN
                new_off[gi] = off
                off += self.slots[gi].numel
            off = start + -(-(off - start) // multiple) * multiple
            ranges[b] = (start, off)
        if sorted(new_off) != list(range(len(self.slots))):
            raise ValueError("relayout: every slot must be in exactly one bucket")
        numel = (off + ALIGN - 1) // ALIGN * ALIGN
        data = torch.zeros(numel, dtype=self.dtype, device=self.device)
        grad = torch.zeros(numel, dtype=self.dtype, device=self.device)
        old_of = {s.index: s.offset for s in self.slots}
        with torch.no_grad():
            for s in self.slots:
                o, n = new_off[s.index], s.numel
                data[o:o + n].copy_(self.data[old_of[s.index]:old_of[s.index] + n])
                grad[o:o + n].copy_(self.grad[old_of[s.index]:old_of[s.index] + n])
        shift = {}
        for s in self.slots:
            shift[s.index] = new_off[s.index] - old_of[s.index]
            s.offset = new_off[s.index]
            s.view = grad[s.offset:s.offset + s.numel]
        for p in self.params:
            s = self.slot_of[id(p)]
            o = self.param_offset[id(p)] + shift[s.index]
            self.param_offset[id(p)] = o
            p.data = data[o:o + p.numel()].view_as(p)
            p.grad = grad[o:o + p.numel()].view_as(p)
        self.data, self.grad, self.numel = data, grad, numel
        if getattr(self, "t_mats", None):
            by_old = {old_of[s.index]: s.index for s in self.slots}
            self.t_mats = sorted((o + shift[by_old[o]] if o in by_old else o, r, c) for o, r, c in self.t_mats)
            self.t_index = {m[0]: i for i, m in enumerate(self.t_mats)}
            self.data_t = None
        return ranges

    # --- views ----------------------------------------------------------------------
    def weight(self, params: Sequence[torch.nn.Parameter], shape: Tuple[int, int]) -> torch.Tensor:
        """Contiguous weight view spanning adjacent params (e.g. wq|wk|wv)."""
        o = self.param_offset[id(params[0])]
        n = 0
        for p in params:
            if self.param_offset[id(p)] != o + n:
                raise ValueError("fused params are not adjacent in the flat buffer")
            n += p.numel()
        return self.data[o:o + n].view(shape)

    def slot(self, p: torch.nn.Parameter) -> GradSlot:
        return self.slot_of[id(p)]

    # --- transposed weight shadows (GPU) ---------------------------------------------------
    # hipBLASLt runs the data-gradient GEMM dX = dY W about 10-15% faster with W supplied
    # K-contiguous, i.e. in the forward GEMM's layout (tools/gemm_bench.py --layouts). Registered
    # matrices keep a transposed copy in ``data_t`` (same offsets), refreshed by the optimizer right
    # after it updates them (same stream, so never stale for the next backward) and by every path
    # that loads parameters (checkpoint load, broadcast, load_state_dict).
    def register_transposed(self, params: Sequence[torch.nn.Parameter], shape: Tuple[int, int]) -> bool:
        rows, cols = shape
        if not self.data.is_cuda or self.data.element_size() != 2 or rows % 64 or cols % 64:
            return False
        o = self.param_offset[id(params[0])]
        if not hasattr(self, "t_mats"):
            self.t_mats: List[Tuple[int, int, int]] = []
            self.t_index: Dict[int, int] = {}
            self.data_t = None
        if o not in self.t_index:
            self.t_index[o] = len(self.t_mats)
            self.t_mats.append((o, rows, cols))
            self.t_mats.sort()
            self.t_index = {m[0]: i for i, m in enumerate(self.t_mats)}
        return True

    def weight_t(self, params: Sequence[torch.nn.Parameter]) -> Optional[torch.Tensor]:
        """[cols, rows] transposed view of a registered fused weight, or None."""
        if not getattr(self, "t_mats", None):
            return None
        o = self.param_offset[id(params[0])]
        i = self.t_index.get(o)
        if i is None:
            return None
        if self.data_t is None:
            self.refresh_transposed()
        _, rows, cols = self.t_mats[i]
        return self.data_t[o:o + rows * cols].view(cols, rows)

    def transposed_in(self, lo: int, hi: int) -> List[Tuple[int, int, int]]:
        """(offset, rows, cols) of the registered matrices starting inside [lo, hi), in offset
        order; the transposed buffer exists afterwards (an optimizer writing the shadows itself)."""
        if not getattr(self, "t_mats", None):
            return []
        if self.data_t is None:
            self.refresh_transposed()
        return [m for m in self.t_mats if lo <= m[0] < hi]

    def refresh_transposed(self, lo: int = 0, hi: Optional[int] = None):
        """Re-derive the transposed copies of registered matrices inside [lo, hi), on the current
        stream (call after anything that writes parameters)."""
        if not getattr(self, "t_mats", None):
            return
        from .. import _ext

        if self.data_t is None:
            self.data_t = torch.empty_like(self.data)
            lo, hi = 0, None
        hi = self.numel if hi is None else hi
        C = _ext.require_for(self.data)
        for o, rows, cols in self.t_mats:
            if lo <= o < hi:
                C.transpose2d(self.data[o:o + rows * cols].view(rows, cols),
                              self.data_t[o:o + rows * cols].view(cols, rows))

    # --- step protocol ----------------------------------------------------------------
    def rebind_grad(self, new: torch.Tensor):
        """Move the gradient space into ``new`` (same numel/dtype/device; e.g. an IPC-exportable
        allocation for the xGMI all-reduce): every ``p.grad`` and slot view is re-pointed."""
        if new.numel() != self.numel or new.dtype != self.grad.dtype or new.device != self.grad.device:
            raise ValueError("rebind_grad: buffer must match the flat gradient buffer")
        self.grad = new
        for p in self.params:
            o = self.param_offset[id(p)]
            p.grad = new[o:o + p.numel()].view_as(p)
        for s in self.slots:
            s.view = new[s.offset:s.offset + s.numel]

    def zero_grad(self):
        for s in self.slots:
            s.fresh = True
            if not s.fused:
                s.view.zero_()
                self._pending_unfused[s.index] = len(s.params)
        if self.reducer is not None:
            self.reducer.reset()

    def next_micro_batch(self):
        """Start another backward into the SAME gradients (gradient accumulation): slots stay
        written, so every producer adds; readiness counting and bucket state start over."""
        for s in self.slots:
            if not s.fused:
                self._pending_unfused[s.index] = len(s.params)
        if self.reducer is not None:
            self.reducer.reset()

    def _make_hook(self, slot: GradSlot) -> Callable:
        def hook(p):
            left = self._pending_unfused.get(slot.index, len(slot.params)) - 1
            self._pending_unfused[slot.index] = left
            slot.fresh = False
            if left == 0:
                self._ready(slot)
        return hook

    def _ready(self, slot: GradSlot):
        if self.reducer is not None:
            self.reducer.mark_ready(slot)

    def state_bytes(self) -> int:
        return self.numel * self.data.element_size()
