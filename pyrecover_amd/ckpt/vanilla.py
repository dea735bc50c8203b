"""Vanilla (single-file) checkpoints: ``ckpt_{step}.pt`` + optional ``.md5`` sidecar.

API and file semantics follow reference pyrecover/checkpoint.py:25-215 (``save_ckpt_vanilla`` /
``load_ckpt_vanilla``): rank 0 writes one ``torch.save``-loadable archive holding
``{epoch, step, model, optimizer, lr_scheduler[, sampler_state]}`` with unprefixed model keys; the
``.md5`` sidecar is the 32-hex md5 of the whole file; ``latest`` resolves to the newest ``*.pt``.

Differences (all compatible with the reference's readers):
* the archive is produced by the C++ engine from a pinned-memory snapshot (async optional), the
  md5 is computed while writing, and the file appears atomically (tmp + fsync + rename);
* a ``pyrecover_state`` entry carries RNG state and run metadata;
* no model-device assert, no per-rank 3 s stagger, numeric retention (D7),
  and ``module.``/``_orig_mod.`` prefixes are stripped on load (D12).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from pathlib import Path
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .. import _ext
from . import core
from .serialization import plan_archive

logger = logging.getLogger("pyrecover")


def _device_of(model) -> torch.device:
    for p in core.unwrap(model).parameters():
        return p.device
    return torch.device("cpu")


def save_ckpt_vanilla(model, optimizer, lr_scheduler=None, sampler=None, step: int = 0, epoch: Optional[int] = None,
                      checkpoint_path: str = "checkpoint.pt", max_keep: int = 3, verify: bool = True,
                      is_distributed: bool = False, rank: int = 0, *, async_save: bool = False, fsync: bool = True,
                      extra_state=None, defer_md5: Optional[bool] = None) -> str:
    """``defer_md5`` (default: on unless PYRECOVER_DEFER_MD5=0): with ``verify`` the whole-file
    ``.md5`` is computed by a background re-read after the archive is durable; False computes it
    inline, so the sidecar exists when the save returns (the time-aware final checkpoint)."""
    if is_distributed:
        dist.barrier()
    core.prepare_optimizer_state(optimizer)  # collective: a sharded optimizer gathers its moments
    rngs = core.gather_rng_states() if is_distributed else None  # collective: every rank's streams
    if rank == 0 or not is_distributed:
        state = core.build_state(model, optimizer, lr_scheduler, sampler, step, epoch, extra_state, rngs)
        ck = core.Checkpointer.get(_device_of(model))
        staged = ck.stage(state)
        prefix = Path(checkpoint_path).name
        if prefix.endswith(".pt"):
            prefix = prefix[:-3]
        records, keep = plan_archive(staged, prefix or "archive")
        base = Path(checkpoint_path).parent

        def done(res, base=base, t0=time.perf_counter()):
            core.apply_retention(base, max_keep, distributed=False)
            md5 = "" if not verify else (", .md5 sidecar pending (background digest)" if res.get("md5_deferred")
                                         else f", md5 {res['md5']}")
            logger.info(f"checkpoint {checkpoint_path}: {res['bytes'] / 2**30:.2f} GiB in {res['seconds']:.2f}s" + md5)

        # The archive and its .md5parts (parallel per-segment MD5s, what our loader verifies) are
        # durable when the job completes; the reference's whole-file .md5 (serial MD5 at ~0.9 GB/s,
        # ~45 s at 7B) follows from a background re-read of the file unless PYRECOVER_DEFER_MD5=0.
        if defer_md5 is None:
            defer_md5 = os.environ.get("PYRECOVER_DEFER_MD5", "1") != "0"
        defer = verify and defer_md5
        if defer:
            core.DEFERRED_MD5_PATHS.add(str(checkpoint_path))
        ck.write(str(checkpoint_path), [("zip", records)], verify, fsync, (staged, keep), done, defer_md5=defer)
        if not async_save:
            ck.wait()
    if is_distributed:
        dist.barrier()
    return str(checkpoint_path)


def verify_checkpoint(path: str) -> Tuple[bool, str]:
    """Compare the file's md5 with its ``.md5`` sidecar (streaming, native; whole file)."""
    try:
        core.flush_all()  # a deferred sidecar of this process lands first
        want = Path(str(path) + ".md5").read_text().strip()
        got = _ext.native().md5_file(str(path))
        if want != got:
            return False, f"Checksum mismatch for checkpoint {path}"
        return True, ""
    except Exception as e:
        return False, str(e)


def load_state_into(model, optimizer, lr_scheduler, sampler, ckpt) -> Tuple[int, int]:
    m = core.unwrap(model)
    sd = core.strip_prefixes(ckpt["model"])
    with torch.no_grad():
        missing, unexpected = m.load_state_dict(sd, strict=False)
    if missing or unexpected:
        raise RuntimeError(f"checkpoint/model key mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
    if optimizer is not None and "optimizer" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer"])
    if lr_scheduler is not None and "lr_scheduler" in ckpt:
        sd = dict(ckpt["lr_scheduler"])
        if hasattr(lr_scheduler, "lr_lambdas"):
            # dcp drops the list of (empty) lambda states when flattening; LambdaLR needs it back
            sd.setdefault("lr_lambdas", [None] * len(sd.get("base_lrs", lr_scheduler.lr_lambdas)))
        lr_scheduler.load_state_dict(sd)
    if sampler is not None and "sampler_state" in ckpt and hasattr(sampler, "load_state_dict"):
        sampler.load_state_dict(ckpt["sampler_state"])
    core.restore_rng_from(ckpt.get("pyrecover_state"))
    return ckpt.get("epoch", 0), ckpt.get("step", 0)


def load_ckpt_vanilla(model, optimizer, lr_scheduler=None, sampler=None, checkpoint_path: str = "latest",
                      experiment_dir: str = ".", verify: bool = True, is_distributed: bool = False,
                      rank: int = 0) -> Tuple[int, int]:
    if is_distributed:
        dist.barrier()
    core.wait_all()
    if checkpoint_path == "latest":
        checkpoint_path = core.get_latest_checkpoint(str(experiment_dir))
        if checkpoint_path is None:
            raise RuntimeError(f"No checkpoint found in {experiment_dir}")
    from . import fastload

    plan = None
    if fastload.ENABLED:
        try:
            plan = fastload.plan_vanilla(str(checkpoint_path), model, optimizer)
        except (ValueError, KeyError, OSError, RuntimeError) as e:  # not an archive the planner maps
            logger.info(f"fast load not applicable ({e}); using torch.load")
    if plan is not None:
        # native parallel read straight into the flat buffers, .md5parts verified on the way
        ckpt, pl = plan
        md5parts = fastload.read_md5parts(str(checkpoint_path)) if verify else None
        if md5parts is not None and md5parts[1] != Path(checkpoint_path).stat().st_size:
            raise RuntimeError(f"Checksum mismatch for checkpoint {checkpoint_path}: size differs from its md5parts")
        stats = fastload.execute(pl, fastload.flat_buffers(model, optimizer), verify, md5parts,
                                 str(checkpoint_path), is_distributed)
        epoch, step = fastload.finish_state(model, optimizer, lr_scheduler, sampler, ckpt, pl)
        del ckpt
        logger.info(f"native read: {stats['bytes_read'] / 2**30:.2f} GiB in {stats['read_s']:.2f}s "
                    f"(verified: {stats['verified']})")
    else:
        result = {"ok": True, "err": ""}
        th = None
        if verify and rank == 0:
            def _v():
                result["ok"], result["err"] = verify_checkpoint(checkpoint_path)
            th = threading.Thread(target=_v, daemon=True)
            th.start()
        ckpt = torch.load(checkpoint_path, map_location="cpu", mmap=True, weights_only=True)
        epoch, step = load_state_into(model, optimizer, lr_scheduler, sampler, ckpt)
        del ckpt
        if th is not None:
            th.join()
            if not result["ok"]:
                raise RuntimeError(result["err"])
    if is_distributed:
        dist.barrier()
    logger.info(f"Checkpoint loaded from {checkpoint_path} (epoch {epoch}, step {step})")
    return epoch, step
