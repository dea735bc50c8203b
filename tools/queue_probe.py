#!/usr/bin/env python
"""Which hardware queue each stream of a training step lands on (1 GPU; SURVEY §5.8, round-5 verdict).

Runs a Llama-2-7B-shape step (fewer layers) with the four kinds of device work a DDP step issues:
compute (forward / backward / GEMMs), the RCCL all-reduce stream (a 1-rank RCCL group, collectives
forced on with PYRECOVER_FORCE_ALLREDUCE=1), the overlapped AdamW side stream, and the asynchronous
checkpoint snapshot (its device-to-device hop into the HBM bounce buffer runs a kernel on the
checkpoint engine's low-priority stream). Record it with

    rocprofv3 --kernel-trace -d gpurun_out/qprobe -o q -- python3 tools/queue_probe.py

and summarise with `python tools/queue_probe.py --summary gpurun_out/qprobe/q_results.db` (or a
kernel-trace CSV): dispatches per (queue, kernel family), and whether two families share a queue.
"""
import argparse
import collections
import os
import sqlite3
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def family(name: str) -> str:
    n = name.lower()
    if "nccl" in n or "rccl" in n or "allreduce" in n:
        return "rccl"
    if "adamw" in n:
        return "adamw"
    if "copy16" in n or "copy1_" in n:
        return "ckpt_snapshot"
    return "compute"


def summary(path: str):
    if path.endswith(".db"):
        rows = sqlite3.connect(path).execute("select name, queue_id from kernels").fetchall()
    else:
        import csv

        rows = [(r["Kernel_Name"], r["Queue_Id"]) for r in csv.DictReader(open(path))]
    by_q = collections.defaultdict(collections.Counter)
    for name, q in rows:
        by_q[q][family(name)] += 1
    print("| queue | dispatches by family |")
    print("|---|---|")
    shared = []
    for q, c in sorted(by_q.items(), key=lambda kv: str(kv[0])):
        print(f"| {q} | {dict(c)} |")
        fams = [f for f in c if f != "compute"] + (["compute"] if c.get("compute") else [])
        if len(fams) > 1:
            shared.append((q, fams))
    print("queues shared by more than one family:", shared if shared else "none")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--summary", default="")
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=4)
    a = ap.parse_args()
    if a.summary:
        summary(a.summary)
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    os.environ["PYRECOVER_FORCE_ALLREDUCE"] = "1"
    import torch
    import torch.distributed as dist

    from pyrecover_amd.ckpt import core as ckcore
    from pyrecover_amd.ckpt.vanilla import save_ckpt_vanilla
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel.ddp import GradReducer
    from pyrecover_amd.parallel.dist import rccl_pg_options

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kw = {"device_id": dev}
    opts = rccl_pg_options()
    if opts is not None:
        kw["pg_options"] = opts
    dist.init_process_group("nccl", rank=0, world_size=1, **kw)
    cfg = get_preset("llama2-7b", seq_len=2048, n_layers=a.layers)
    torch.manual_seed(0)
    with torch.device(dev):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.bfloat16)
        model = Transformer(cfg)
        torch.set_default_dtype(prev)
    flat = model.flatten_(tokens_per_step=a.batch * 2048)
    red = GradReducer(flat, bucket_cap_mb=256.0)
    assert red.force_collective
    opt = FlatAdamW(flat, lr=1e-5, fused=True)
    opt.enable_overlap(red)
    opt.pre_update_fences.append(ckcore.fence_all)
    d = tempfile.mkdtemp(prefix="qprobe_")
    for step in range(1, a.steps + 1):
        t = torch.randint(0, cfg.vocab_size, (a.batch, 2049), device=dev)
        opt.zero_grad()
        model(t[:, :-1], labels=t[:, 1:]).backward()
        red.finish()
        ckcore.fence_all()
        opt.step()
        if step == 2:  # asynchronous save: the snapshot's D2D hop runs beside the next step
            save_ckpt_vanilla(model, opt, None, None, step, 1, os.path.join(d, f"ckpt_{step}.pt"), max_keep=1,
                              verify=False, async_save=True)
    torch.cuda.synchronize()
    ckcore.wait_all()
    dist.destroy_process_group()
    print("queue probe done:", d)


if __name__ == "__main__":
    main()
