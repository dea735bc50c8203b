"""What does a large device-to-host copy on a side stream cost the training step running beside it?

Builds the bench model (default Llama-2-7B shape, batch 2), times one step alone, then one step
while N GiB are copied D2H into pinned memory on a low-priority stream (the checkpoint snapshot's
second hop), with the copy issued as ONE hipMemcpyAsync per 256 MiB chunk. Run it under
`rocprofv3 --kernel-trace --memory-copy-trace` to see whether the copies run on the DMA engines or
as blit kernels on the CUs.

    python tools/d2h_overlap_probe.py [--gib 37.7] [--model llama2-7b] [--batch 2]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=37.7)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=2048)
    a = ap.parse_args()
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel.ddp import GradReducer

    dev = torch.device("cuda", 0)
    cfg = get_preset(a.model, seq_len=a.seq_len)
    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        m = Transformer(cfg)
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    red = GradReducer(flat)
    opt = FlatAdamW(flat, lr=1e-5)
    opt.enable_overlap(red)
    g = torch.Generator(device=dev)
    g.manual_seed(1)

    def step():
        t = torch.randint(0, cfg.vocab_size, (a.batch, a.seq_len + 1), device=dev, generator=g)
        opt.zero_grad()
        m(t[:, :-1], labels=t[:, 1:]).backward()
        red.finish()
        opt.step()

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for _ in range(2):
        step()
    base = [timed(step) for _ in range(3)]
    nbytes = int(a.gib * 2**30)
    src = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    lo, _ = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, 0)
    side = torch.cuda.Stream(device=dev, priority=0)
    chunk = 256 << 20

    def copy_all():
        with torch.cuda.stream(side):
            for o in range(0, nbytes, chunk):
                n = min(chunk, nbytes - o)
                dst[o:o + n].copy_(src[o:o + n], non_blocking=True)

    copy_alone = timed(lambda: (copy_all(), side.synchronize()))
    res = {"step_s": [round(x, 4) for x in base], "copy_alone_s": round(copy_alone, 4),
           "copy_gbps": round(nbytes / copy_alone / 1e9, 1)}

    def overlapped():
        copy_all()
        step()
        side.synchronize()

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    copy_all()
    step()
    torch.cuda.current_stream().synchronize()
    res["step_beside_copy_s"] = round(time.perf_counter() - t0, 4)
    side.synchronize()
    res["both_done_s"] = round(time.perf_counter() - t0, 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
