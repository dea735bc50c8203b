"""One GEMM kernel run a few times, for rocprofv3 --pmc passes (tools/gemm_prof.sh):

    python tools/gemm_pmc.py --kernel nt|nt32|wgrad|lib --m 32768 --n 12288 --k 4096 [--iters 5]

nt/nt32: C.gemm_nt_ (x [m, k], w [n, k]); wgrad: C.wgrad_mm_ (dy [k, m]^T x [k, n], i.e. M=m);
lib: torch.mm(x, w.t()). Random uniform [-1, 1) bf16 operands."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="nt")
    ap.add_argument("--m", type=int, default=32768)
    ap.add_argument("--n", type=int, default=12288)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning("auto")  # lib: the step's tuned hipBLASLt solution table
    C = _ext.native()
    dev = torch.device("cuda", 0)

    def rnd(*s):
        return (torch.rand(*s, device=dev) * 2 - 1).bfloat16()
    if a.kernel == "nt32":
        os.environ["PRA_GEMM_NT_KB"] = "32"
    if a.kernel.startswith("nt") or a.kernel == "lib":
        x, w = rnd(a.m, a.k), rnd(a.n, a.k) * 0.05
        y = torch.empty(a.m, a.n, device=dev, dtype=torch.bfloat16)
        f = (lambda: torch.mm(x, w.t(), out=y)) if a.kernel == "lib" else (lambda: C.gemm_nt_(x, w, y))
    else:
        dy, x = rnd(a.k, a.m) * 0.05, rnd(a.k, a.n)
        y = torch.empty(a.m, a.n, device=dev, dtype=torch.bfloat16)
        f = lambda: C.wgrad_mm_(dy, x, y, False)  # noqa: E731
    for _ in range(a.iters):
        f()
    torch.cuda.synchronize()
    print("done", a.kernel)


if __name__ == "__main__":
    main()
