#!/usr/bin/env python
"""Interleaved in-process A/B of attention kernel choices (pyrecover_amd._ext.set_attn_options;
rounds alternate, medians reported), on random data. Every arm's outputs are compared with the
first arm's: o and lse for --fwd, dq/dk/dv for the backward.

  python tools/attn_ab.py --opt dkdv_impl --values 0,1 [--B 16 --S 2048 --Hq 32 --Hkv 32]
  python tools/attn_ab.py --fwd --opt fwd_pipe --values 0,1
"""
import argparse
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--opt", required=True, choices=["fwd_pipe", "fwd_thr", "dkdv_impl", "dq_pipe", "dkdv_split", "dkdv_kreg"])
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fwd", action="store_true", help="time the forward instead")
    ap.add_argument("--set", default="", help="fixed OPT=VAL[,OPT=VAL] for every arm")
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    fixed = dict(kv.split("=", 1) for kv in filter(None, a.set.split(",")))
    _ext.set_attn_options(**{k: float(v) for k, v in fixed.items()})
    dev = torch.device("cuda", 0)
    B, S, Hq, Hkv, D = a.B, a.S, a.Hq, a.Hkv, a.D
    g = torch.Generator(device=dev).manual_seed(0)
    qkv = torch.randn(B * S, (Hq + 2 * Hkv) * D, device=dev, generator=g).bfloat16()
    q = qkv[:, :Hq * D].view(B, S, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].view(B, S, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:].view(B, S, Hkv, D)
    scale = 1 / math.sqrt(D)
    o, lse = C.attn_fwd(q, k, v, scale, True)
    do = torch.randn(B, S, Hq, D, device=dev, generator=g).bfloat16()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    vals = a.values.split(",")
    times = {x: [] for x in vals}
    outs = {}

    def run():
        if a.fwd:
            return C.attn_fwd(q, k, v, scale, True)
        C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True)
        return dq, dk, dv

    def select(x):
        _ext.set_attn_options(**{a.opt: float(x)})

    for x in vals:  # warm + results
        select(x)
        res = run()
        torch.cuda.synchronize()
        outs[x] = tuple(t.clone() for t in res)
    for _ in range(a.rounds):
        for x in vals:
            select(x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[x].append(e0.elapsed_time(e1) / a.iters)
    ref = outs[vals[0]]
    names = ("o", "lse") if a.fwd else ("dq", "dk", "dv")
    for x in vals:
        diffs = ", ".join(f"{n} {(u.float() - w.float()).abs().max().item():.3g}"
                          for n, u, w in zip(names, outs[x], ref))
        print(f"{a.opt}={x}: median {statistics.median(times[x]):.4f} ms  min {min(times[x]):.4f} ms  "
              f"max|d - {vals[0]}|: {diffs}", flush=True)


if __name__ == "__main__":
    main()
