"""Weight-gradient GEMM dW = dY^T X on row-major activations (K = tokens): the hand-written MFMA
kernel (csrc/kernels/gemm_wgrad.hip, C.wgrad_mm_) against hipBLASLt in the layouts the step can use:
  nt      torch.mm(dY.t(), X)                         (no copies; library on K-slow operands)
  tn      torch.mm(dYt, Xt.t()) on pre-transposed copies (the library's fast layout, copies free)
  tn+T    the two HIP transposes + tn                 (what the default step pays)
  hip     C.wgrad_mm_(dY, X, out)
Checks hip against an fp32 reference first. Rounds interleaved in one process (rule: A/B in one
process); prints one JSON line per shape with median us and TFLOP/s.

    python tools/wgrad_bench.py [--tokens 32768] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402

# (name, M = out features, N = in features) of the 7B step's weight gradients
SHAPES = [("qkv", 12288, 4096), ("o", 4096, 4096), ("w13", 22016, 4096), ("w2", 4096, 11008)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--dims", default="", help="name:M:N[,...] instead of the 7B shapes (e.g. GPT-2-medium "
                    "qkv:3072:1024,o:1024:1024,w13:5632:1024)")
    args = ap.parse_args()
    global SHAPES
    if args.dims:
        SHAPES = [(n, int(m), int(k)) for n, m, k in (d.split(":") for d in args.dims.split(","))]
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")  # the library arms use the step's tuned solution table
    C = _ext.native()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # correctness: fp32 reference on a short K, plain and accumulate
    for name, M, N in SHAPES:
        K = 512
        dy = torch.randn(K, M, device=dev).bfloat16()
        x = torch.randn(K, N, device=dev).bfloat16()
        ref = dy.float().t() @ x.float()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        C.wgrad_mm_(dy, x, out, False)
        err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
        c0 = torch.randn(M, N, device=dev).bfloat16()
        out2 = c0.clone()
        C.wgrad_mm_(dy, x, out2, True)
        err2 = (out2.float() - (ref + c0.float())).abs().max().item() / ref.abs().max().item()
        print(json.dumps({"check": name, "rel_err": err, "rel_err_acc": err2}), flush=True)
        assert err < 1e-2 and err2 < 1e-2, (name, err, err2)
    T = args.tokens
    sel = set(args.shapes.split(",")) if args.shapes else None
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, M, N in SHAPES:
        if sel and name not in sel:
            continue
        dy = (torch.rand(T, M, device=dev) * 2 - 1).bfloat16()
        x = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
        dyT = dy.t().contiguous()
        xT = x.t().contiguous()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        arms = {
            "nt": lambda: torch.mm(dy.t(), x, out=out),
            "tn": lambda: torch.mm(dyT, xT.t(), out=out),
            "tn+T": lambda: torch.mm(C.transpose2d(dy, dyT), C.transpose2d(x, xT).t(), out=out),
            "hip": lambda: C.wgrad_mm_(dy, x, out, False),
        }
        res = {k: [] for k in arms}
        for _ in range(args.rounds):
            for k, fn in arms.items():
                for _ in range(2):
                    fn()
                s.record()
                for _ in range(args.iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                res[k].append(s.elapsed_time(e) * 1e3 / args.iters)
        flops = 2.0 * M * N * T
        print(json.dumps({"shape": name, "M": M, "N": N, "K": T,
                          **{k: {"us": round(statistics.median(v), 1),
                                 "TF": round(flops / statistics.median(v) / 1e6, 1)} for k, v in res.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
