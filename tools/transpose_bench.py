"""Isolated throughput of the 16-bit 2-D transpose (csrc/kernels/elementwise.hip) on the shapes the
7B / Llama-3-8B steps transpose: activations [tokens, dim] for the TN weight gradients and the
weight shadows [out, in]. Prints effective HBM bandwidth (read + write bytes / time).

    python tools/transpose_bench.py                 # register kernel (default)
    PYRECOVER_TRANSPOSE=lds python tools/transpose_bench.py   # LDS-tiled kernel
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402

SHAPES = [(16384, 4096), (16384, 11008), (12288, 4096), (22016, 4096), (4096, 11008), (8192, 4096)]


def main():
    C = _ext.native()
    dev = torch.device("cuda", 0)
    variant = os.environ.get("PYRECOVER_TRANSPOSE", "reg")
    for R, Cc in SHAPES:
        x = torch.randn(R, Cc, device=dev).bfloat16()
        out = torch.empty(Cc, R, device=dev, dtype=x.dtype)
        for _ in range(3):
            C.transpose2d(x, out)
        torch.cuda.synchronize()
        assert torch.equal(out, x.t().contiguous())
        n = 20
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            C.transpose2d(x, out)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / n
        s.record()
        for _ in range(n):
            out.copy_(x.t())
        e.record()
        torch.cuda.synchronize()
        us_torch = s.elapsed_time(e) * 1e3 / n
        gb = 2 * x.numel() * 2 / 1e9
        print(json.dumps({"variant": variant, "shape": [R, Cc], "us": round(us, 1),
                          "TBps": round(gb / us * 1e3, 2),
                          "torch_copy_us": round(us_torch, 1)}), flush=True)
    # transposing epilogues at the 7B shapes (T = 16384 tokens, F = 11008, QKV width 12288)
    T, F = 16384, 11008
    gu = torch.randn(T, 2 * F, device=dev).bfloat16()
    dy = torch.randn(T, F, device=dev).bfloat16()
    x = torch.randn(T, 3 * 4096, device=dev).bfloat16()
    tab = torch.randn(2048, 64, 2, device=dev)
    cases = [("swiglu_fwd_t", lambda: C.swiglu_fwd_t(gu), 2 * T * F * 2 + 2 * T * F * 2),
             ("swiglu_bwd_t", lambda: C.swiglu_bwd_t_(dy, gu), T * F * 2 + 3 * 2 * T * F * 2),
             ("rope_t", lambda: C.rope_t_(x, 2 * 4096, tab, 128, 2048, True), 3 * x.numel() * 2)]
    for name, fn, nbytes in cases:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        n = 20
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / n
        print(json.dumps({"variant": variant, "kernel": name, "us": round(us, 1),
                          "TBps": round(nbytes / 1e9 / us * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
