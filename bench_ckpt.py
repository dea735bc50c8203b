#!/usr/bin/env python
"""Checkpoint save + resume wall-clock (second half of the BASELINE.json headline metric).

Builds the bench model (default Llama-2-7B-shape, bf16, random init) on one GPU, runs a
training step so the AdamW moments are populated, then measures for each format:

* vanilla sync:   ``save_ckpt_vanilla`` until it returns: the archive and its ``.md5parts`` are
                  durable (``vanilla_save_s``); the reference's whole-file ``.md5`` sidecar follows
                  from a background digest (``vanilla_md5_sidecar_s``, measured from the same start;
                  ``PYRECOVER_DEFER_MD5=0`` makes the save itself wait for it);
* vanilla async:  the training-visible stall (snapshot staged, writer launched) and the
                  background completion time, with a training step running in between;
* sharded:        ``save_ckpt_distributed`` (dcp-compatible directory) sync;
* resume:         load time for each format into a fresh model/optimizer, verifying bit equality.

Prints one JSON line. ``--dir`` should point at node-local storage (NVMe); sizes are reported.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import torch


def _wstats(core):
    last = core.WRITE_STATS.get("last", {})
    return {k: (round(v, 3) if isinstance(v, float) else v) for k, v in last.items() if k not in ("error", "md5")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--n-layers", type=int, default=None)
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--dir", default="/tmp/pyrecover_ckpt_bench")
    ap.add_argument("--verify", action="store_true", help="write + check the .md5 sidecar")
    ap.add_argument("--formats", default="vanilla,async,sharded")
    args = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pyrecover_amd.ckpt import core, fastload
    from pyrecover_amd.ckpt.sharded import load_ckpt_distributed, save_ckpt_distributed
    from pyrecover_amd.ckpt.vanilla import load_ckpt_vanilla, save_ckpt_vanilla, verify_checkpoint
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler
    from pyrecover_amd.parallel.ddp import GradReducer

    dev = torch.device("cuda", 0)
    cfg = get_preset(args.model, seq_len=args.seq_len, n_layers=args.n_layers)

    def build():
        torch.manual_seed(0)
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.bfloat16)
        with torch.device(dev):
            m = Transformer(cfg)
        torch.set_default_dtype(prev)
        flat = m.flatten_()
        red = GradReducer(flat)
        opt = FlatAdamW(flat, lr=1e-5)
        opt.enable_overlap(red)
        opt.pre_update_fences.append(core.fence_all)
        return m, flat, red, opt, build_lr_scheduler(opt, 10)

    model, flat, red, opt, sched = build()
    g = torch.Generator(device=dev)
    g.manual_seed(1)

    def step():
        t = torch.randint(0, cfg.vocab_size, (args.batch, args.seq_len + 1), device=dev, generator=g)
        opt.zero_grad()
        model(t[:, :-1], labels=t[:, 1:]).backward()
        red.finish()
        opt.step()
        sched.step()

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step()
    torch.cuda.synchronize()
    step_s = time.perf_counter() - t0

    shutil.rmtree(args.dir, ignore_errors=True)
    os.makedirs(args.dir, exist_ok=True)
    out = {"metric": "checkpoint save+resume wall-clock", "model": f"{args.model}-shape",
           "params": model.num_params(), "state_bytes": opt.checkpoint_bytes(), "step_s": round(step_s, 3),
           "dir": args.dir, "whole_file_md5": os.environ.get("PYRECOVER_WHOLE_MD5", "1") != "0"}
    ref_params = flat.data.clone()
    ref_v = opt.exp_avg_sq.clone()
    formats = args.formats.split(",")

    def check_loaded(tag):
        m2, flat2, _, opt2, sched2 = build()
        return m2, flat2, opt2, sched2

    if "vanilla" in formats:
        p = os.path.join(args.dir, "ckpt_2.pt")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        save_ckpt_vanilla(model, opt, sched, None, 2, 1, p, max_keep=0, verify=args.verify)
        out["vanilla_save_s"] = round(time.perf_counter() - t0, 3)
        out["vanilla_write"] = _wstats(core)
        if args.verify:  # the reference's whole-file .md5 sidecar lands from a background digest
            core.flush_all()
            out["vanilla_md5_sidecar_s"] = round(time.perf_counter() - t0, 3)
            out["vanilla_md5_sidecar_ok"] = verify_checkpoint(p)[0]
        out["vanilla_file_gib"] = round(os.path.getsize(p) / 2**30, 3)
        del model, opt
        torch.cuda.empty_cache()
        m2, flat2, opt2, sched2 = check_loaded("vanilla")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        load_ckpt_vanilla(m2, opt2, sched2, None, p, verify=args.verify)
        torch.cuda.synchronize()
        out["vanilla_load_s"] = round(time.perf_counter() - t0, 3)
        out["vanilla_load_native"] = {k: (round(v, 3) if isinstance(v, float) else v)
                                      for k, v in fastload.LAST_STATS.items()}
        out["vanilla_bit_exact"] = bool(torch.equal(flat2.data, ref_params) and torch.equal(opt2.exp_avg_sq, ref_v))
        model, flat, opt, sched = m2, flat2, opt2, sched2
        red = GradReducer(flat)
        opt.enable_overlap(red)
        opt.pre_update_fences.append(core.fence_all)
        os.remove(p)
        if os.path.exists(p + ".md5"):
            os.remove(p + ".md5")

    if "async" in formats:
        p = os.path.join(args.dir, "ckpt_3.pt")
        # as train.py --async-checkpoint does: the pinned pool is allocated before training runs,
        # so the first save does not pay for it
        core.Checkpointer.get(flat.data.device).prewarm(int(opt.checkpoint_bytes() * 1.05) + (64 << 20),
                                                        background=False)
        step()
        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        save_ckpt_vanilla(model, opt, sched, None, 3, 1, p, max_keep=0, verify=args.verify, async_save=True)
        out["async_stall_s"] = round(time.perf_counter() - t0, 3)
        t1 = time.perf_counter()
        step()  # training continues while the snapshot drains and the file is written
        # the compute stream only: a device-wide synchronize would also wait for the snapshot's
        # D2H drain on the checkpoint engine's own stream, which training never waits for
        torch.cuda.current_stream(dev).synchronize()
        out["async_overlapped_step_s"] = round(time.perf_counter() - t1, 3)
        out["async_snapshot_two_hop"] = bool(core.Checkpointer.get(dev).engine.last_two_hop())
        core.wait_all()
        out["async_total_s"] = round(time.perf_counter() - t0, 3)
        os.remove(p)
        if os.path.exists(p + ".md5"):
            os.remove(p + ".md5")

    if "sharded" in formats:
        ref_params = flat.data.clone()
        ref_v = opt.exp_avg_sq.clone()
        d = os.path.join(args.dir, "ckpt_4")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        save_ckpt_distributed(model, opt, sched, None, 4, 1, d, max_keep=0)
        out["sharded_save_s"] = round(time.perf_counter() - t0, 3)
        out["sharded_write"] = _wstats(core)
        del model, opt
        torch.cuda.empty_cache()
        m2, flat2, opt2, sched2 = check_loaded("sharded")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        load_ckpt_distributed(m2, opt2, sched2, None, d)
        torch.cuda.synchronize()
        out["sharded_load_s"] = round(time.perf_counter() - t0, 3)
        out["sharded_load_native"] = {k: (round(v, 3) if isinstance(v, float) else v)
                                      for k, v in fastload.LAST_STATS.items()}
        out["sharded_bit_exact"] = bool(torch.equal(flat2.data, ref_params) and torch.equal(opt2.exp_avg_sq, ref_v))
        shutil.rmtree(d, ignore_errors=True)

    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
