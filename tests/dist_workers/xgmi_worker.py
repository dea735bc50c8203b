"""Worker for tests/test_xgmi_gpu.py: 2+ ranks (torchrun), all pinned to one GPU
(PYRECOVER_LOCAL_DEVICE=0, PYRECOVER_DIST_BACKEND=gloo). Trains llama-tiny for a few steps with
the chosen all-reduce backend and writes rank 0's flat parameters + a direct all-reduce check."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["rccl", "xgmi"], required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--overlap", action="store_true")
    a = ap.parse_args()
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel import dist as D
    from pyrecover_amd.parallel.ddp import GradReducer, broadcast_flat

    lrank, world = D.maybe_init_distributed(True)
    rank = D.get_rank()
    dev = torch.device("cuda", D.gpu_index(lrank))
    torch.manual_seed(0)
    cfg = get_preset("llama-tiny", seq_len=256)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        m = Transformer(cfg)
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    broadcast_flat(flat)
    red = GradReducer(flat, bucket_cap_mb=0.5, first_bucket_mb=0.25, backend=a.backend)
    assert red.num_buckets > 3
    # 1) direct all-reduce check on rank-dependent data
    g = torch.Generator(device=dev)
    g.manual_seed(100 + rank)
    flat.grad.copy_(torch.randn(flat.numel, generator=g, device=dev).to(flat.grad.dtype))
    expect = torch.zeros(flat.numel, dtype=torch.float32, device=dev)
    for r in range(world):
        gr = torch.Generator(device=dev)
        gr.manual_seed(100 + r)
        expect += torch.randn(flat.numel, generator=gr, device=dev).to(flat.grad.dtype).float()
    for b in range(red.num_buckets):
        red._launch(b)
    red.next_to_launch = red.num_buckets
    red.finish()
    red.reset()
    torch.cuda.synchronize()
    direct_err = (flat.grad.float() - expect.to(flat.grad.dtype).float()).abs().max().item()
    # 2) training steps
    opt = FlatAdamW(flat, lr=1e-3, grad_scale=1.0 / world)
    if a.overlap:
        opt.enable_overlap(red)
    gen = torch.Generator(device=dev)
    gen.manual_seed(123 + rank)
    for _ in range(3):
        t = torch.randint(0, cfg.vocab_size, (2, 257), device=dev, generator=gen)
        opt.zero_grad()
        m(t[:, :-1], labels=t[:, 1:]).backward()
        red.finish()
        opt.step()
        red.reset()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({"params": flat.data.cpu(), "direct_err": direct_err}, a.out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
