#!/usr/bin/env python
"""SwiGLU backward kernel A/B at the 7B B16 shape (T = 32768 tokens, F = 11008), in place over gu
as in the training step; arms interleaved per round, medians reported with the achieved HBM rate
(bytes: read g, u, dy; write dg, du).

  python tools/swiglu_bwd_bench.py [--T 32768 --F 11008 --variants 0,1,2]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=32768)
    ap.add_argument("--F", type=int, default=11008)
    ap.add_argument("--variants", default="0,1,2")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from pyrecover_amd import _ext

    C = _ext.native()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    gu0 = torch.randn(a.T, 2 * a.F, device=dev, generator=g).bfloat16()
    dy = torch.randn(a.T, a.F, device=dev, generator=g).bfloat16()
    gu = gu0.clone()
    vals = [int(x) for x in a.variants.split(",")]
    ref = C.swiglu_bwd(dy, gu0, None, 0)
    for v in vals:  # in place (the step's form) must equal the out-of-place grid-stride result
        gu.copy_(gu0)
        C.swiglu_bwd(dy, gu, gu, v)
        assert torch.equal(gu, ref), v
    nbytes = 5 * a.T * a.F * 2
    times = {v: [] for v in vals}
    for _ in range(a.rounds):
        for v in vals:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                C.swiglu_bwd(dy, gu, gu, v)  # values drift (in place); the work is identical
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    for v in vals:
        med = statistics.median(times[v])
        print(f"variant {v}: median {med:.4f} ms  min {min(times[v]):.4f} ms  {nbytes / med / 1e9:.2f} TB/s",
              flush=True)


if __name__ == "__main__":
    main()
