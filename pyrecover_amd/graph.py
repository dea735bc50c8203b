"""HIP-graph capture of the whole training step: ``train.py --compile``.

The reference compiles the model with ``torch.compile(model, fullgraph=True)`` (reference
train.py:103-105), which on its hardware means Inductor/Triton kernels. Here the hot ops are
already fused HIP kernels, so what is left to remove is per-launch CPU overhead. This module
captures one complete step (forward, backward with the gradient-bucket hooks, RCCL reduction and
the flat AdamW, including the side-stream overlapped updates) into one hipGraph
(``torch.cuda.CUDAGraph`` is hipGraph on ROCm) and replays it for every later step.

What changes per step without re-capture:
* the batch is copied into the graph's static input tensors;
* learning rate and Adam bias corrections are uploaded to device memory
  (:meth:`FlatAdamW.begin_graph_step`) and read by the optimizer kernel;
* checkpoint snapshot fences are applied to the stream *before* the replay (a captured graph
  cannot wait on an event recorded outside it), so a step never overtakes an in-flight
  checkpoint copy.
Everything host-side (logging, time-aware stop, checkpoint scheduling, data loading) stays
outside the graph. Shapes are static (fixed batch and sequence length), as in the reference.
"""
from __future__ import annotations

import os

import torch


def capture_allowed(world_size: int) -> tuple:
    """Whether the step may be captured with ``world_size`` ranks: ``(ok, reason)``.

    One rank: always. Several ranks: the backward's bucket all-reduces would be captured into the
    graph. Gloo collectives run on the host and cannot be captured at all; RCCL collectives can be
    captured, but replaying them has not been validated on a multi-GPU node, so capture stays off
    unless ``PYRECOVER_GRAPH_COLLECTIVES=1`` opts in. Callers run the step eagerly otherwise."""
    if world_size <= 1:
        return True, ""
    import torch.distributed as dist

    backend = dist.get_backend() if dist.is_initialized() else None
    if backend != "nccl":
        return False, f"backend {backend!r} collectives cannot be captured into a HIP graph"
    if os.environ.get("PYRECOVER_GRAPH_COLLECTIVES", "0") != "1":
        return False, ("HIP-graph capture of RCCL collectives is not validated on multi-GPU runs "
                       "(set PYRECOVER_GRAPH_COLLECTIVES=1 to capture them anyway)")
    return True, ""


class StepGraph:
    def __init__(self, model, optimizer, reducer=None, fences=None, pre_step=None):
        self.model = model
        self.opt = optimizer
        self.reducer = reducer
        self.fences = list(fences or [])
        self.pre_step = pre_step  # device-side work between backward and the update (grad clipping)
        self.graph = None
        self.static_x = None
        self.static_y = None
        self.loss = None
        self.replays = 0

    @property
    def captured(self) -> bool:
        return self.graph is not None

    def _eager_body(self):
        loss = self.model(self.static_x, labels=self.static_y)
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        if self.pre_step is not None:
            self.pre_step()
        self.opt.step()
        return loss

    def _capture(self, x, y):
        self.static_x = x.detach().clone()
        self.static_y = y.detach().clone()
        self.opt.enable_graph_mode()
        self.opt.begin_graph_step()
        self.opt.zero_grad()  # host-side "fresh" flags decide which kernels get recorded
        saved = self.opt.pre_update_fences
        self.opt.pre_update_fences = []  # applied before each replay instead
        torch.cuda.synchronize()
        torch.cuda.empty_cache()  # eager-step blocks are not reusable by the graph's private pool
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g):
                self.loss = self._eager_body()
        finally:
            self.opt.pre_update_fences = saved
        self.graph = g

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Run one training step on batch (x, y); returns the (static) loss tensor."""
        if self.graph is None:
            self._capture(x, y)  # capture records but does not execute: replay below runs it
        else:
            self.static_x.copy_(x, non_blocking=True)
            self.static_y.copy_(y, non_blocking=True)
            self.opt.begin_graph_step()
        for f in self.fences:
            f()
        self.graph.replay()
        self.replays += 1
        return self.loss
