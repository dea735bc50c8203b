"""Does the row stride of the weight-gradient GEMM's operands change its rate? dW = dY^T X on the
MFMA kernel (C.wgrad_mm_) with dY [T, M] stored at row strides M, M + 64, M + 128, ... (views of a
wider buffer), arms interleaved in one process, median of rounds. The W1|W3 shape (M = 22016) runs
0.90x of the QKV / O shapes' rate in the step; this separates the shape from the stride.

    python tools/wgrad_ld_probe.py [--tokens 32768] [--pads 0,64,128,256,512]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--pads", default="0,64,128,256,512")
    ap.add_argument("--shapes", default="w13:22016:4096,qkv:12288:4096")
    a = ap.parse_args()
    C = _ext.native()
    dev = torch.device("cuda", 0)
    T = a.tokens
    pads = [int(p) for p in a.pads.split(",")]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for spec in a.shapes.split(","):
        name, M, N = spec.split(":")
        M, N = int(M), int(N)
        x = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
        src = (torch.rand(T, M, device=dev) * 2 - 1).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        arms = {}
        ref = None
        for p in pads:
            dy = torch.empty(T, M + p, device=dev, dtype=torch.bfloat16)[:, :M]
            dy.copy_(src)
            arms[p] = dy
            C.wgrad_mm_(dy, x, out, False)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            else:
                assert torch.equal(ref, out), f"stride {M + p} changed the result"
        res = {p: [] for p in pads}
        for _ in range(a.rounds):
            for p, dy in arms.items():
                C.wgrad_mm_(dy, x, out, False)
                s.record()
                for _ in range(a.iters):
                    C.wgrad_mm_(dy, x, out, False)
                e.record()
                torch.cuda.synchronize()
                res[p].append(s.elapsed_time(e) * 1e3 / a.iters)
        flops = 2.0 * M * N * T
        print(json.dumps({"shape": name, "M": M, "N": N, "K": T,
                          **{f"ld{M + p}": {"us": round(statistics.median(v), 1),
                                            "TF": round(flops / statistics.median(v) / 1e6, 1)}
                             for p, v in res.items()}}), flush=True)
        del x, src, out, arms


if __name__ == "__main__":
    main()
