#!/usr/bin/env python
"""Same-process A/B of whole training steps (bench.py's 7B B16 step: forward, backward, overlapped
AdamW), arms alternating round by round on one model, so box-to-box clock differences cancel.

An arm is `name:module.ATTR=value;module.ATTR=value` over pyrecover_amd modules (values are Python
literals), applied before its steps and undone after them, e.g.

    python tools/step_ab.py --arm "tile:ops.fused.SWIGLU_BWD_VARIANT=-1" \
                            --arm "grid:ops.fused.SWIGLU_BWD_VARIANT=0" [--rounds 4 --steps 5]

Prints the median ms/step per arm and the per-round values (JSON lines).
"""
import argparse
import ast
import importlib
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_arm(spec):
    """`opt.ATTR=value` sets an attribute of the optimizer instance; `attn.OPTION=value` an
    attention kernel option (_ext.set_attn_options); `native.SETTER=value` calls that setter of the
    extension before the arm's steps and with 0 after them; the item `noupdate` skips the AdamW update
    kernels (a diagnostic arm: what the optimizer costs the step)."""
    name, _, body = spec.partition(":")
    sets = []
    for item in filter(None, body.split(";")):
        if item.strip() == "noupdate":
            sets.append(("opt", "_update_range", "noupdate"))
            continue
        lhs, _, rhs = item.partition("=")
        mod, _, attr = lhs.strip().rpartition(".")
        if mod in ("attn", "native"):  # attention option / native setter C.<attr>(value), reset to 0 after
            sets.append((mod, attr, ast.literal_eval(rhs.strip())))
            continue
        target = "opt" if mod == "opt" else importlib.import_module("pyrecover_amd." + mod)
        sets.append((target, attr, ast.literal_eval(rhs.strip())))
    return name, sets


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arm", action="append", required=True)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch-per-gpu", type=int, default=16)
    a = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel.ddp import GradReducer

    arms = [parse_arm(s) for s in a.arm]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = get_preset(a.model, seq_len=a.seq_len)
    torch.manual_seed(1234)
    with torch.device(dev):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.bfloat16)
        model = Transformer(cfg)
        torch.set_default_dtype(prev)
    flat = model.flatten_(tokens_per_step=a.batch_per_gpu * a.seq_len)
    reducer = GradReducer(flat, bucket_cap_mb=256.0)
    opt = FlatAdamW(flat, lr=1e-5, fused=True)
    opt.enable_overlap(reducer)
    B, S = a.batch_per_gpu, a.seq_len
    gen = torch.Generator(device=dev)
    gen.manual_seed(0)

    def step():
        t = torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=gen)
        opt.zero_grad()
        loss = model(t[:, :-1], labels=t[:, 1:])
        loss.backward()
        reducer.finish()
        opt.step()
        return loss

    from pyrecover_amd import _ext

    def resolve(sets):
        out = []
        for m, k, v in sets:
            if m in ("attn", "native"):
                continue
            m = opt if m == "opt" else m
            if v == "noupdate":
                v = lambda *args, **kw: None  # noqa: E731
            out.append((m, k, v))
        return out

    def run(arm, n):
        attn = {k: v for m, k, v in arm[1] if m == "attn"}
        prev_attn = _ext.set_attn_options(**attn) if attn else None
        natives = [(k, v) for m, k, v in arm[1] if m == "native"]
        for k, v in natives:
            getattr(_ext.native(), k)(v)
        sets = resolve(arm[1])
        old = [(m, k, m.__dict__[k] if k in m.__dict__ else getattr(m, k)) for m, k, _ in sets]
        for m, k, v in sets:
            setattr(m, k, v)
        try:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                loss = step()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1000 / n, float(loss.item())
        finally:
            for k, _ in natives:
                getattr(_ext.native(), k)(0)
            if prev_attn is not None:
                _ext.set_attn_options(**prev_attn)
            for m, k, v in old:
                if m is opt and k == "_update_range":
                    del m.__dict__[k]  # back to the class method
                else:
                    setattr(m, k, v)

    for arm in arms:
        run(arm, a.warmup)
    per = {arm[0]: [] for arm in arms}
    for r in range(a.rounds):
        order = arms if r % 2 == 0 else arms[::-1]
        for arm in order:
            ms, loss = run(arm, a.steps)
            per[arm[0]].append(ms)
            print(json.dumps({"round": r, "arm": arm[0], "ms_per_step": round(ms, 2), "loss": round(loss, 4)}),
                  flush=True)
    base = statistics.median(per[arms[0][0]])
    for name, v in per.items():
        med = statistics.median(v)
        print(json.dumps({"arm": name, "median_ms_per_step": round(med, 2), "min": round(min(v), 2),
                          "tokens_per_s": round(B * S * 1000 / med, 1),
                          "vs_first_pct": round(100 * (med / base - 1), 2)}), flush=True)


if __name__ == "__main__":
    main()
