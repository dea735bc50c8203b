#!/usr/bin/env python
"""Isolated bandwidth of the AdamW update kernels on one weight matrix (csrc/kernels/optim.hip):
the flat streaming kernel (p, g, m, v: 14 B per element) against the tiled kernel that also writes
the transposed weight shadow (16 B per element), exact and fast math. (Round 6 used it to pick the
non-temporal, two-chunks-per-thread schedule and 128 x 128 transposing tiles: profiles/r6/adamw/.)

    python tools/adamw_bench.py [--rows 28672 --cols 4096 --iters 20]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=28672)
    ap.add_argument("--cols", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    dev = torch.device("cuda", 0)
    R, K = a.rows, a.cols
    p = torch.randn(R, K, device=dev).bfloat16()
    g = torch.randn(R, K, device=dev).bfloat16() * 1e-3
    m = torch.zeros(R, K, device=dev, dtype=torch.bfloat16)
    v = torch.zeros(R, K, device=dev, dtype=torch.bfloat16)
    pt = torch.empty(K, R, device=dev, dtype=torch.bfloat16)
    hp = dict(lr=1e-4, b1=0.9, b2=0.95, eps=1e-8, wd=0.1, bc1=0.1, bc2_sqrt=0.2236, gscale=1.0)
    cases = {
        "flat": (lambda f: C.adamw_flat_(p.view(-1), g.view(-1), m.view(-1), v.view(-1), fast=f, **hp), 14),
        "t": (lambda f: C.adamw_t_(p, g, m, v, pt, fast=f, **hp), 16),
    }
    out = {}
    for name, (fn, bpe) in cases.items():
        for fast in (False, True):
            for _ in range(3):
                fn(fast)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn(fast)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            key = f"{name}_{'fast' if fast else 'exact'}"
            out[key] = {"ms": round(ms, 4), "TB_per_s": round(R * K * bpe / ms / 1e9, 2)}
            print(json.dumps({key: out[key]}), flush=True)
    print(json.dumps({"rows": R, "cols": K, "results": out}), flush=True)


if __name__ == "__main__":
    main()
