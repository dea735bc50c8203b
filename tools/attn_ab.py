#!/usr/bin/env python
"""Interleaved in-process A/B of attention backward variants selected by an environment variable
read per call (rounds alternate; medians reported), on random data.

  python tools/attn_ab.py --var PRA_ATTN_DELTA_PRE --values 0,1 [--B 16 --S 2048 --Hq 32 --Hkv 32]
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
    ap.add_argument("--var", required=True)
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--B", type=int, default=16)
    ap.add_argument("--S", type=int, default=2048)
    ap.add_argument("--Hq", type=int, default=32)
    ap.add_argument("--Hkv", type=int, default=32)
    ap.add_argument("--D", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--fwd", action="store_true", help="time the forward instead")
    ap.add_argument("--set", default="", help="fixed VAR=VAL[,VAR=VAL] for every arm")
    a = ap.parse_args()
    for kv in filter(None, a.set.split(",")):
        k_, v_ = kv.split("=", 1)
        os.environ[k_] = v_
    from pyrecover_amd import _ext

    C = _ext.native()
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
            C.attn_fwd(q, k, v, scale, True)
        else:
            C.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, scale, True)

    for x in vals:  # warm + results
        os.environ[a.var] = x
        run()
        torch.cuda.synchronize()
        outs[x] = (dq.clone(), dk.clone(), dv.clone())
    for _ in range(a.rounds):
        for x in vals:
            os.environ[a.var] = x
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[x].append(e0.elapsed_time(e1) / a.iters)
    ref = outs[vals[0]]
    for x in vals:
        diff = max(((u.float() - w.float()).abs().max().item() for u, w in zip(outs[x], ref)))
        print(f"{a.var}={x}: median {statistics.median(times[x]):.4f} ms  min {min(times[x]):.4f} ms  "
              f"max|d - {vals[0]}| {diff:.3g}", flush=True)


if __name__ == "__main__":
    main()
