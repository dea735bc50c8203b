#!/usr/bin/env python
"""Isolated bandwidth of the 16-bit 2-D transpose (csrc/kernels/elementwise.hip transpose_reg_kernel,
the TN weight-gradient operands at small batch) against a plain device copy of the same bytes. (Round 6: 5.0-6.5 TB/s, at the copy's rate; two or
four tiles per wave were no faster: profiles/r6/transpose/.)

    python tools/transpose_bench.py [--shapes 2048x4096,2048x6144,4096x14336,32768x4096]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2048x4096,2048x6144,4096x14336,32768x4096")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    for shp in a.shapes.split(","):
        R, K = (int(x) for x in shp.split("x"))
        x = torch.randn(R, K, device="cuda").bfloat16()
        out = torch.empty(K, R, device="cuda", dtype=torch.bfloat16)
        cp = torch.empty_like(x)
        assert torch.equal(C.transpose2d(x), x.t())
        t_ms = timed(lambda: C.transpose2d(x, out), a.iters)
        res = {"transpose_us": round(t_ms * 1e3, 2)}
        c_ms = timed(lambda: cp.copy_(x), a.iters)
        nb = 2 * x.numel() * 2
        print(json.dumps({"shape": shp, **res, "transpose_TBps": round(nb / t_ms / 1e9, 2),
                          "copy_us": round(c_ms * 1e3, 2), "copy_TBps": round(nb / c_ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
