#!/usr/bin/env python
"""Where the weight-gradient GEMM's main loop loses time: the kernel with its main-loop LDS-DMA
removed (exp 1), its fragment reads removed (exp 2), both (exp 3), against the real kernel (exp 0)
and hipBLASLt on the K-contiguous layout. Timing only -- exp 1..3 compute garbage.

    python tools/gemm_exp.py [--M 32768 --N 4096 --K 16384]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=16384)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")
    C = _ext.native()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    M, N, K = a.M, a.N, a.K
    dy = torch.randn(K, M, device=dev, generator=g).bfloat16()
    x = torch.randn(K, N, device=dev, generator=g).bfloat16()
    dyt, xt = dy.t().contiguous(), x.t().contiguous()
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, generator=g).bfloat16()
    xa = torch.randn(M, K, device=dev, generator=g).bfloat16()
    arms = {"lib_tn": lambda: torch.mm(dyt, xt.t()), "lib_nt": lambda: torch.mm(xa, w.t()),
            "nt": lambda: C.gemm_nt_(xa, w, y)}
    for e in range(4):
        arms[f"exp{e}"] = (lambda e=e: C.wgrad_mm_exp_(dy, x, y, e))
    t = {k: [] for k in arms}
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, f in arms.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                f()
            e.record()
            e.synchronize()
            t[name].append(s.elapsed_time(e) / a.iters)
    for name in arms:
        med = statistics.median(t[name])
        print(f"{name:7s} {med:8.4f} ms  {2 * M * N * K / med / 1e9:7.1f} TF", flush=True)


if __name__ == "__main__":
    main()
