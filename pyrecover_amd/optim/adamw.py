"""AdamW over the flat parameter space, state_dict-compatible with ``torch.optim.AdamW``.

The reference builds ``torch.optim.AdamW(model.parameters(), lr, fused=--fused-optimizer)``
(reference train.py:120-122) with default betas/eps/weight_decay on all params and bf16 states
(no fp32 master copy). :class:`FlatAdamW` keeps that contract (same param_groups keys, per-param
``state[i] = {"step", "exp_avg", "exp_avg_sq"}`` in ``model.parameters()`` order), but the moments
live in two flat buffers laid out like the flat parameters, and the update is one HIP kernel
over the whole model (``pra_adamw_flat``: fp32 opmath, torch ``_fused_adamw_`` semantics).

``master_weights=True`` (``--master-weights fp32``; SURVEY §8 D18: "keep pure-bf16 as the default for
parity, optional fp32 master"): the update runs on an fp32 master copy of the parameters with fp32
moments (``pra_adamw_master``), and the 16-bit parameters the model computes with are the master
rounded once after every update. The master is saved as a third per-parameter state tensor
(``state[i]["master_param"]``) next to the fp32 moments; a checkpoint without it (pure-bf16 runs,
the reference's) resumes with the master taken from the loaded parameters.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from .. import _ext
from ..ops import sched
from ..parallel.flat import FlatParams

# Matrices with a transposed weight shadow (parallel/flat.py) are updated by a tiled AdamW kernel
# that writes the shadow from the values it just computed (no transpose pass re-reading the
# weights); False (from code: tests, A/B tools) falls back to flat AdamW + a separate transpose.
FUSED_T = True
# When an overlapped bucket update is enqueued on the side stream (PYRECOVER_OPT_SCHED):
#   "attn" (default): held until the next attention backward, then enqueued behind an event recorded
#            between its dQ and dK/dV kernels (ops.sched.attention_window), so it runs beside dK/dV,
#            which leaves room on every CU and reads little from HBM;
#   "eager": as soon as the bucket is reduced (it then lands beside the register-bound dQ kernel and
#            the memory-bound SwiGLU backward and slows them).
# Same-process A/B (profiles/r3/step_ab_attnwin_*.log): 7B B16 1063.3 -> 1056.5 ms, 7B B1 99.6 ->
# 97.9 ms, Llama-3-8B S8192 B1 373.3 -> 361.5 ms, GPT-2-medium unchanged; no update at all: 1043.9
# ms at B16. (Holding the updates for the W1|W3 / QKV data-gradient GEMMs instead measured +1.45%.)
# Until a window has been seen, a bucket is held for at most one bucket: when the next bucket is
# reduced and no attention window released the held ones (a model whose attention takes the torch
# path -- fp64, head_dim not 64/128 -- or has no attention), they are enqueued then, so the update
# still overlaps the backward instead of running serialized in step().
OPT_SCHED = os.environ.get("PYRECOVER_OPT_SCHED", "attn")
# PYRECOVER_ADAMW_FAST (default 0): torch _fused_adamw_'s exact expression tree (mixed fp64/fp32,
# correctly rounded divisions; bit-equal to the reference's --fused-optimizer). 1: the
# hardware reciprocal / square root in pure fp32 (csrc/kernels/optim.hip adamw_elem<FAST>, ~17
# instead of ~60 VALU per element beside the attention backward; 7B B1 98.5 -> 97.2 ms, B16 within
# noise, profiles/r3/step_ab_fast_*.log), whose p differs from torch's by a few fp32 ulps.
FAST_MATH = os.environ.get("PYRECOVER_ADAMW_FAST", "0") == "1"


class FlatAdamW(torch.optim.AdamW):
    def __init__(self, flat: FlatParams, params=None, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, fused: Optional[bool] = None, grad_scale: float = 1.0,
                 master_weights: bool = False):
        # default order = the model's parameters() order when the model recorded it (the
        # reference's optimizer-state indices), else the flat buffer order
        params = list(params) if params is not None else list(getattr(flat, "module_order", None) or flat.params)
        for p in params:
            if id(p) not in flat.param_offset:
                raise ValueError("every optimized parameter must live in the flat buffer")
        # fused=None keeps torch from validating device support for the CPU path; the flag is
        # recorded in param_groups for state_dict parity with the reference.
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        for g in self.param_groups:
            g["fused"] = bool(fused)
        if len(self.param_groups) != 1:
            raise ValueError("FlatAdamW supports a single param group (the reference uses one)")
        self.flat = flat
        flat.layout_frozen = True  # the moments below are laid out like the flat buffers
        self.grad_scale = grad_scale  # e.g. 1/world_size after a SUM all-reduce
        self.grad_scale_dev: Optional[torch.Tensor] = None  # device-side multiplier (clipping)
        # fp32 master + fp32 moments for 16-bit parameters (fp32 / fp64 models already update in place)
        self.master: Optional[torch.Tensor] = None
        if master_weights and flat.data.element_size() == 2:
            self.master = flat.data.float()
        sdt = torch.float32 if self.master is not None else flat.data.dtype
        self.exp_avg = torch.zeros(flat.data.shape, dtype=sdt, device=flat.data.device)
        self.exp_avg_sq = torch.zeros(flat.data.shape, dtype=sdt, device=flat.data.device)
        self._step = 0
        self._bind_state()
        self.overlap = False
        self._in_step = False
        self._done_ranges = []
        self._held = []  # (bucket, lo, hi, work) of reduced buckets not yet enqueued (OPT_SCHED "attn")
        self._gathers = []  # parameter all-gathers issued behind the updates (sharded optimizer)
        self._window_seen = False  # an attention window released held buckets (HIP attention path)
        self.pre_update_fences = []  # callables run on the update stream before any update
        # graph mode (train.py --compile): step-dependent scalars come from device memory
        self.graph_mode = False
        self.hyper: Optional[torch.Tensor] = None
        self._hyper_ring = []
        self._hyper_slot = 0

    # --- captured-step (HIP graph) support ---------------------------------------------------
    def enable_graph_mode(self):
        """Kernels read {lr, bc1, bc2_sqrt} from ``self.hyper`` (device fp64[3]) instead of
        launch arguments, and the host step counter advances in :meth:`begin_graph_step`, so one
        captured step replays correctly at every later step and learning rate."""
        if not self.flat.data.is_cuda:
            raise RuntimeError("graph mode needs the parameters on a GPU")
        self.graph_mode = True
        dev = self.flat.data.device
        self.hyper = torch.zeros(3, dtype=torch.float64, device=dev)
        # pinned staging ring: a slot is rewritten only after its previous H2D copy completed
        self._hyper_ring = [(torch.zeros(3, dtype=torch.float64).pin_memory(), torch.cuda.Event()) for _ in range(4)]

    def begin_graph_step(self):
        """Host side of one replayed step: advance the step count and upload the scalars."""
        self._step += 1
        lr, _, _, _, _, bc1, bc2_sqrt = self._coeffs()
        host, ev = self._hyper_ring[self._hyper_slot]
        self._hyper_slot = (self._hyper_slot + 1) % len(self._hyper_ring)
        ev.synchronize()
        host[0], host[1], host[2] = lr, bc1, bc2_sqrt
        self.hyper.copy_(host, non_blocking=True)
        ev.record()

    # --- overlapped update (optimizer-in-backward) ----------------------------------------
    def enable_overlap(self, reducer):
        """Update each gradient bucket as soon as it is reduced, on a side stream, overlapped with
        the rest of the backward pass. Math and result are identical to :meth:`step`."""
        self.overlap = True
        self.reducer = reducer
        reducer.hooks.append(self._on_bucket)
        self.stream = torch.cuda.Stream(device=self.flat.data.device) if self.flat.data.is_cuda else None
        dev = self.flat.data.device
        sched.add_attention_window_hook(self.release_held, dev.index if dev.type == "cuda" else None)

    def _coeffs(self):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        lr, eps, wd = float(g["lr"]), float(g["eps"]), float(g["weight_decay"])
        return lr, b1, b2, eps, wd, 1.0 - b1 ** self._step, math.sqrt(1.0 - b2 ** self._step)

    def _update_range(self, lo, hi, coeffs=None):
        f = self.flat
        lr, b1, b2, eps, wd, bc1, bc2_sqrt = coeffs if coeffs is not None else self._coeffs()
        if not _ext.hip(f.data):
            self._step_reference(lr, b1, b2, eps, wd, bc1, bc2_sqrt, lo, hi)
            return
        C = _ext.require_for(f.data)
        args = (lr, b1, b2, eps, wd, bc1, bc2_sqrt, self.grad_scale, self.grad_scale_dev, self.hyper)
        m, v = self.exp_avg, self.exp_avg_sq

        fast = FAST_MATH
        sharded = self._sharded()
        if self.master is not None:
            # fp32 master update, then the transposed shadows of the matrices in range from the
            # rounded parameters (same stream: the next backward sees them; sharded: after the gather)
            C.adamw_master_(f.data[lo:hi], self.master[lo:hi], f.grad[lo:hi], m[lo:hi], v[lo:hi], *args, fast)
            if not sharded:
                f.refresh_transposed(lo, hi)
            return
        if sharded:
            # an owned chunk cuts matrices: plain update; the shadows are re-derived from the gathered
            # parameters (step)
            C.adamw_flat_(f.data[lo:hi], f.grad[lo:hi], m[lo:hi], v[lo:hi], *args, fast)
            return

        def flat_update(a, b):
            if a < b:
                C.adamw_flat_(f.data[a:b], f.grad[a:b], m[a:b], v[a:b], *args, fast)

        mats = f.transposed_in(lo, hi) if FUSED_T else []
        cur = lo
        rest = []
        for o, rows, cols in mats:
            n = rows * cols
            if o + n > hi:  # (buckets align to fusion groups; kept for safety)
                rest.append(o)
                continue
            flat_update(cur, o)
            sl = slice(o, o + n)
            C.adamw_t_(f.data[sl].view(rows, cols), f.grad[sl].view(rows, cols), m[sl].view(rows, cols),
                       v[sl].view(rows, cols), f.data_t[sl].view(cols, rows), *args, fast)
            cur = o + n
        flat_update(cur, hi)
        if not FUSED_T:
            f.refresh_transposed(lo, hi)  # same stream: the next backward sees the new weights
        for o in rest:
            f.refresh_transposed(o, o + 1)

    def _on_bucket(self, b, lo, hi, work):
        if not self.overlap or self.grad_scale_dev is not None:
            return  # clipping needs the global norm first: fall back to step()
        if not self._in_step:
            self._in_step = True
            if not self.graph_mode:  # graph mode: begin_graph_step() counts the step
                self._step += 1
        if self.stream is None:
            if work is not None:
                work.wait()
            self._update_bucket(b, lo, hi)
            return
        if self._held and not self._window_seen:
            # no attention window has released held buckets yet: this model's backward may offer
            # none, so do not wait any longer than one bucket
            self.release_held()
        self._held.append((b, lo, hi, work))
        if OPT_SCHED != "attn":
            self.release_held()

    def release_held(self, event=None):
        """Enqueue the held bucket updates on the side stream behind `event` (default: one recorded
        on the compute stream now). Every read of their weights was enqueued before the bucket was
        published, so any later point of the compute stream is safe."""
        if event is not None:
            self._window_seen = True  # called from an attention window of this device
        if not self._held:
            return
        if event is None:
            event = torch.cuda.Event()
            event.record()
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(event)
            for b, lo, hi, work in self._held:
                if work is not None:
                    work.wait()  # update stream waits for the bucket's all-reduce
                for fence in self.pre_update_fences:
                    fence()
                self._update_bucket(b, lo, hi)
        self._held = []

    # --- sharded optimizer (GradReducer(shard=True), --shard-optimizer) ----------------------
    def _sharded(self) -> bool:
        r = getattr(self, "reducer", None) or getattr(self.flat, "reducer", None)
        return bool(r is not None and r.shard)

    def _update_bucket(self, b, lo, hi, coeffs=None):
        """Update bucket b's parameters this rank owns, then (sharded) all-gather them, issued on the
        current stream behind the update."""
        r = getattr(self.flat, "reducer", None)
        if r is None or not r.shard:
            self._update_range(lo, hi, coeffs)
            self._done_ranges.append((lo, hi))
            return
        for a, z in r.owned(b):
            self._update_range(a, z, coeffs)
            self._done_ranges.append((a, z))
        self._gathers.extend(r.gather_params(b))

    def _finish_gathers(self):
        """The current stream waits for the parameter all-gathers; the transposed shadows are then
        re-derived from the gathered parameters."""
        if not self._gathers and not self._sharded():
            return
        for w in self._gathers:
            w.wait()
        self._gathers = []
        self.flat.refresh_transposed()

    def gather_state(self):
        """Collective (sharded optimizer): all-gather the moments (and the fp32 master) so every rank
        holds the full optimizer state, as a checkpoint stores it. A no-op otherwise."""
        r = getattr(self.flat, "reducer", None)
        if r is None or not r.shard:
            return
        if self.overlap and self.stream is not None:
            torch.cuda.current_stream(self.flat.data.device).wait_stream(self.stream)
        ts = [self.exp_avg, self.exp_avg_sq] + ([self.master] if self.master is not None else [])
        works = [w for b in range(r.num_buckets) for w in r.gather_params(b, ts)]
        for w in works:
            w.wait()

    def _bind_state(self):
        for p in self.param_groups[0]["params"]:
            o = self.flat.param_offset[id(p)]
            n = p.numel()
            self.state[p] = {
                "step": torch.tensor(float(self._step), dtype=torch.float32),
                "exp_avg": self.exp_avg[o:o + n].view(p.shape),
                "exp_avg_sq": self.exp_avg_sq[o:o + n].view(p.shape),
            }
            if self.master is not None:
                self.state[p]["master_param"] = self.master[o:o + n].view(p.shape)

    # --- torch.optim.Optimizer API ------------------------------------------------------
    def zero_grad(self, set_to_none: bool = True):
        """Marks gradient slots fresh; the flat gradient views are never set to None."""
        self.flat.zero_grad()
        if self.overlap and self.stream is not None:
            # the next backward overwrites gradients the update stream may still be reading
            torch.cuda.current_stream(self.flat.data.device).wait_stream(self.stream)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.overlap and self.grad_scale_dev is None:
            self.reducer.finish()  # launches (and so updates) any bucket not yet ready
            if not self._in_step and not self.graph_mode:  # no bucket fired (no backward this step)
                self._step += 1
            self.release_held()
            if self.stream is not None:
                torch.cuda.current_stream(self.flat.data.device).wait_stream(self.stream)
            self._finish_gathers()
            self._in_step = False
            self._done_ranges = []
            return loss
        g = self.param_groups[0]
        if not self.graph_mode:
            self._step += 1
        b1, b2 = g["betas"]
        lr, eps, wd = float(g["lr"]), float(g["eps"]), float(g["weight_decay"])
        bc1 = 1.0 - b1 ** self._step
        bc2_sqrt = math.sqrt(1.0 - b2 ** self._step)
        coeffs = (lr, b1, b2, eps, wd, bc1, bc2_sqrt)
        r = getattr(self.flat, "reducer", None)
        if r is not None and r.shard:
            for b, (lo, hi) in enumerate(r.ranges):
                self._update_bucket(b, lo, hi, coeffs)
            self._done_ranges = []
            self._finish_gathers()
            return loss
        self._update_range(0, self.flat.numel, coeffs)
        return loss

    def _step_reference(self, lr, b1, b2, eps, wd, bc1, bc2_sqrt, lo=0, hi=None):
        f = self.flat
        hi = f.numel if hi is None else hi
        gs = self.grad_scale * (float(self.grad_scale_dev[0]) if self.grad_scale_dev is not None else 1.0)
        # `.data`: the update must not bump the flat buffer's autograd version counter (shared by
        # every parameter view), or an overlapped bucket update during backward would invalidate
        # weights other layers saved for their backward (the HIP kernels write through pointers)
        pd, gd, md, vd = f.data.data[lo:hi], f.grad[lo:hi], self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi]
        ct = torch.promote_types(pd.dtype, torch.float32)  # fp32 opmath; fp64 models stay fp64
        p = (self.master[lo:hi] if self.master is not None else pd).to(ct)
        gr = gd.to(ct) * gs
        m = md.to(ct)
        v = vd.to(ct)
        p.mul_(1 - lr * wd)
        m.lerp_(gr, 1 - b1)
        v.mul_(b2).addcmul_(gr, gr, value=1 - b2)
        denom = v.sqrt().div_(bc2_sqrt).add_(eps)
        p.addcdiv_(m, denom, value=-(lr / bc1))
        if self.master is not None:
            self.master[lo:hi].copy_(p)
        pd.copy_(p)
        md.copy_(m)
        vd.copy_(v)

    # --- checkpoint compatibility -------------------------------------------------------
    def checkpoint_bytes(self) -> int:
        """Tensor bytes a checkpoint of this model + optimizer holds: the parameters, both moments
        and (``--master-weights fp32``) the fp32 master -- 6 B/param pure bf16, 14 B/param with the
        master. Sizes the time-aware final-save estimate and the pinned staging pool."""
        n = self.flat.data.nbytes + self.exp_avg.nbytes + self.exp_avg_sq.nbytes
        return n + (self.master.nbytes if self.master is not None else 0)

    def state_dict(self):
        for st in self.state.values():
            st["step"] = torch.tensor(float(self._step), dtype=torch.float32)
        return super().state_dict()

    def load_state_dict(self, state_dict, tensors_loaded: bool = False):
        """Accepts torch.optim.AdamW state dicts (ours or the reference's). ``tensors_loaded``:
        the moments were already written into the flat buffers (native resume path), so only the
        hyper-parameters and step counts are taken from ``state_dict``."""
        groups = state_dict["param_groups"]
        if len(groups) != 1:
            raise ValueError("expected exactly one param group")
        params = self.param_groups[0]["params"]
        saved_ids = groups[0]["params"]
        if len(saved_ids) != len(params):
            raise ValueError(f"optimizer state has {len(saved_ids)} params, model has {len(params)}")
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = v
        steps = set()
        with torch.no_grad():
            for sid, p in zip(saved_ids, params):
                st = state_dict["state"].get(sid, state_dict["state"].get(str(sid)))
                mine = self.state[p]
                if "master_param" in mine and (st is None or "master_param" not in st or not tensors_loaded):
                    # a checkpoint without a master (pure-bf16 run, the reference's): take the loaded
                    # parameters; with one, its fp32 values
                    src = st.get("master_param") if st is not None else None
                    mine["master_param"].copy_(src if src is not None else p.detach())
                if st is None:
                    if not tensors_loaded:
                        mine["exp_avg"].zero_()
                        mine["exp_avg_sq"].zero_()
                    continue
                if not tensors_loaded:
                    mine["exp_avg"].copy_(st["exp_avg"])
                    mine["exp_avg_sq"].copy_(st["exp_avg_sq"])
                steps.add(float(st["step"]))
        if len(steps) > 1:
            raise ValueError(f"inconsistent per-parameter step counts {sorted(steps)}")
        self._step = int(steps.pop()) if steps else 0
        for st in self.state.values():
            st["step"] = torch.tensor(float(self._step), dtype=torch.float32)
