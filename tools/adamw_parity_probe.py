"""Where does the flat AdamW kernel differ from torch._fused_adamw_? One step from a random state
(fp32 and bf16), mismatch counts per tensor, and up to 4096 mismatching elements with their inputs
and both outputs saved for offline analysis of the expression tree (gpurun_out/adamw_probe.pt)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrecover_amd import _ext  # noqa: E402


def main():
    C = _ext.native()
    dev = torch.device("cuda")
    out = {}
    lr, b1, b2, eps, wd = 1e-3, 0.9, 0.999, 1e-8, 0.01
    for dtype in (torch.float32, torch.bfloat16):
        for s in (1, 3):
            torch.manual_seed(7 + s)
            n = 1 << 22
            p = torch.randn(n, device=dev).to(dtype)
            g = (torch.randn(n, device=dev) * 1e-2).to(dtype)
            m = (torch.randn(n, device=dev) * 1e-3).to(dtype) if s > 1 else torch.zeros(n, device=dev, dtype=dtype)
            v = (torch.rand(n, device=dev) * 1e-5).to(dtype) if s > 1 else torch.zeros(n, device=dev, dtype=dtype)
            a = [t.clone() for t in (p, m, v)]
            b = [t.clone() for t in (p, m, v)]
            C.adamw_flat_(a[0], g, a[1], a[2], lr, b1, b2, eps, wd, 1 - b1 ** s, math.sqrt(1 - b2 ** s), 1.0, None,
                          None, False)
            step = torch.full((), float(s), device=dev)
            torch._fused_adamw_([b[0]], [g], [b[1]], [b[2]], [], [step], amsgrad=False, lr=lr, beta1=b1, beta2=b2,
                                weight_decay=wd, eps=eps, maximize=False)
            key = f"{str(dtype).split('.')[-1]}_s{s}"
            bad = (a[0] != b[0]) | (a[1] != b[1]) | (a[2] != b[2])
            print(key, "p", int((a[0] != b[0]).sum()), "m", int((a[1] != b[1]).sum()), "v",
                  int((a[2] != b[2]).sum()), "of", n, flush=True)
            idx = bad.nonzero().flatten()[:4096]
            out[key] = {k: t[idx].float().cpu() for k, t in
                        (("p", p), ("g", g), ("m", m), ("v", v), ("p_ours", a[0]), ("m_ours", a[1]), ("v_ours", a[2]),
                         ("p_torch", b[0]), ("m_torch", b[1]), ("v_torch", b[2]))}
            out[key]["raw"] = {k: t[idx].cpu() for k, t in (("p", p), ("g", g), ("m", m), ("v", v), ("p_torch", b[0]),
                                                           ("m_torch", b[1]), ("v_torch", b[2]), ("p_ours", a[0]))}
    os.makedirs("gpurun_out", exist_ok=True)
    torch.save(out, "gpurun_out/adamw_probe.pt")


if __name__ == "__main__":
    main()
