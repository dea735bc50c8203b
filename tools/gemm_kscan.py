#!/usr/bin/env python
"""Fixed vs per-K cost of the hand-written GEMMs and hipBLASLt: C[M][N] over K = 1k..16k at one
M x N (default 32768 x 4096, 8 rounds of 256 tiles), least-squares fit t(K) = a + b K per kernel.
`a` is the per-launch fixed cost (prologue + epilogue of every tile round + launch), `b` the
steady-state main-loop rate. Arms interleaved, median of rounds, random data.

    python tools/gemm_kscan.py [--M 32768 --N 4096 --ks 1024,2048,4096,8192,16384]
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
    ap.add_argument("--ks", default="1024,2048,4096,8192,16384")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")
    C = _ext.native()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    ks = [int(k) for k in a.ks.split(",")]
    M, N = a.M, a.N
    res = {}
    for K in ks:
        x = torch.randn(M, K, device=dev, generator=g).bfloat16()
        w = torch.randn(N, K, device=dev, generator=g).bfloat16()
        dy = torch.randn(K, M, device=dev, generator=g).bfloat16()  # wgrad: out[M][N] = dy^T xx
        xx = torch.randn(K, N, device=dev, generator=g).bfloat16()
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        arms = {
            "lib_nt": lambda: torch.mm(x, w.t()),
            "nt": lambda: C.gemm_nt_(x, w, y),
            "wgrad": lambda: C.wgrad_mm_(dy, xx, y, False),
        }
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
            res.setdefault(name, []).append((K, med))
            print(f"K={K:6d} {name:7s} {med:8.4f} ms  {2 * M * N * K / med / 1e9:7.1f} TF", flush=True)
        del x, w, dy, xx, y
    for name, pts in res.items():
        n = len(pts)
        mk = sum(k for k, _ in pts) / n
        mt = sum(v for _, v in pts) / n
        b = sum((k - mk) * (v - mt) for k, v in pts) / sum((k - mk) ** 2 for k, _ in pts)
        a0 = mt - b * mk
        print(f"{name:7s} fit: fixed {a0 * 1000:.1f} us per launch, steady {2 * M * N / b / 1e9:.1f} TF", flush=True)


if __name__ == "__main__":
    main()
