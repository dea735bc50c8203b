#!/usr/bin/env python
"""Headline benchmark: DDP training throughput at seq_len=2048, bf16, on 1..8 MI355X.

Measures the reference's headline metric (tokens/sec at seq 2048 bf16, BASELINE.json) on the
Llama-2-7B-shape transformer of BASELINE.json config 3 (dim 4096, 32 layers, 32 heads, SwiGLU
11008, vocab 32000), random-init weights, synthetic token data. Each timed step is a full
training step: forward, backward with bucketed RCCL gradient all-reduce (N>1), fused AdamW
update and LR-scheduler step -- nothing is skipped.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched by
``torch.distributed.run`` (one rank per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from env).
Rank 0 prints ONE JSON line; ``value`` is the whole-job aggregate tokens/s (max time over ranks).

Started as ``python bench.py --gpus N`` (N>1) WITHOUT a rank environment, this process touches no
GPU: it starts ``torch.distributed.run`` with N ranks as a child process on 127.0.0.1 and exits
with its code. A rank whose process group does not have exactly N ranks exits non-zero, and the
JSON line reports ``ranks_seen`` (the process group's size) next to ``n_gpus``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _bucket_arg(v):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pyrecover_amd.parallel.bucket_tune import parse_bucket_arg

    return parse_bucket_arg(v)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="llama2-7b")
    ap.add_argument("--seq-len", type=int, default=2048)
    ap.add_argument("--batch-per-gpu", type=int, default=16)
    ap.add_argument("--bucket-mb", type=_bucket_arg, default=256.0,
                    help="all-reduce bucket MiB, or 'auto' (startup probe: parallel/bucket_tune.py)")
    ap.add_argument("--master-weights", choices=["none", "fp32"], default="none",
                    help="fp32 master weights + moments (default none: pure bf16, as the reference)")
    ap.add_argument("--lr", type=float, default=1e-5)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--profile-steps", type=int, default=0, help="emit roctx ranges for this many steps")
    ap.add_argument("--no-overlap-optimizer", action="store_true",
                    help="AdamW after backward instead of per bucket during backward")
    ap.add_argument("--allreduce", choices=["rccl", "xgmi"], default="rccl",
                    help="gradient all-reduce: RCCL (default) or the direct per-link xGMI backend")
    ap.add_argument("--graph", action="store_true",
                    help="capture the step into a HIP graph after the warmup steps (train.py --compile)")
    ap.add_argument("--phase-timing", action="store_true",
                    help="record device events around forward / backward / optimizer of each timed step")
    ap.add_argument("--no-comm-timing", action="store_true",
                    help="W > 1: skip the per-bucket collective timing (events; no host sync in the step)")
    ap.add_argument("--shard-optimizer", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                    help="W > 1: ZeRO-1 (reduce-scatter, 1/W AdamW update, parameter all-gather; train.py flag); "
                         "auto: for models without transposed weight shadows at this batch; a bare flag means on")
    ap.add_argument("--sparse-embedding-grad", choices=["auto", "on", "off"], default="auto",
                    help="W > 1: token-embedding gradient as (id, row) pairs (auto: tokens per step <= vocab / 2)")
    ap.add_argument("--comm-probe", choices=["rccl", "all", "off"], default="rccl",
                    help="W > 1, after the timed steps: all-reduce probe bus bandwidth on the job's group "
                         "(rccl; all: also the direct xGMI engine) reported in the JSON line")
    ap.add_argument("--cpu", action="store_true",
                    help="run on the CPU over gloo (tests of the launcher and the DDP path; not a benchmark)")
    ap.add_argument("--gemm-tuning", choices=["auto", "off", "tune"], default="auto",
                    help="hipBLASLt solution table (tuning/): auto = use the committed table if present")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, gpus: int, env) -> list:
    """The child command that runs this benchmark with ``gpus`` ranks, or [] when this process is
    already a rank (a torchrun/SLURM environment) or ``gpus`` is 1."""
    if gpus <= 1 or "WORLD_SIZE" in env or "SLURM_PROCID" in env and int(env.get("SLURM_NTASKS", "1")) > 1:
        return []
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)


def _gemm_sites(tokens, dim):
    """Which GEMM sites of this step run the hand-written MFMA kernels (ops/fused.py site rules)."""
    from pyrecover_amd.ops import fused

    nt_auto = tokens >= fused.NT_AUTO_MIN_TOKENS and dim >= fused.NT_AUTO_MIN_K
    nt = sorted(fused.GEMM_SITES) if (not fused.GEMM_AUTO or nt_auto) else []
    # weight-gradient sites also need one 256x256 output tile per CU (decided per GEMM at run time)
    wg = sorted(fused.WGRAD_SITES) if (not fused.WGRAD_AUTO or tokens >= fused.WGRAD_AUTO_MIN_TOKENS) else []
    return {"nt_with_epilogues": nt, "weight_gradient_candidates": wg}


def _adamw_fast() -> bool:
    from pyrecover_amd.optim import adamw

    return adamw.FAST_MATH


def _opt_sched(tokens: int = 0) -> str:
    """Where the overlapped AdamW update runs; `tokens` = B * S of one attention call (the window
    opens before the dQ kernel at <= 4096 tokens unless the attention option bwd_window pins it)."""
    from pyrecover_amd import _ext
    from pyrecover_amd.optim import adamw

    if adamw.OPT_SCHED == "attn":
        w = _ext._attn_opts.get("bwd_window", -1)
        early = w == 1 or (w < 0 and 0 < tokens <= 4096)
        return "beside the attention dQ and dK/dV kernels" if early else "beside the attention dK/dV kernels"
    return {"eager": "per bucket as reduced"}.get(adamw.OPT_SCHED, adamw.OPT_SCHED)


def main():
    args = parse()
    cmd = launch_command(sys.argv[1:], args.gpus, os.environ)
    if cmd:
        # no GPU call has happened in this process: the ranks are fresh children
        import subprocess

        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(cmd, env=env))
    root = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, root)
    from pyrecover_amd.utils.gemm_tuning import configure_gemm_tuning

    configure_gemm_tuning(args.gemm_tuning)
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler
    from pyrecover_amd.parallel import dist as D
    from pyrecover_amd.parallel.ddp import GradReducer, broadcast_flat, comm_env
    from pyrecover_amd.utils.flops import num_flop_per_token

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    if world_env > 1:
        lrank, world = D.maybe_init_distributed(True)
    else:
        lrank, world = 0, 1
    ranks_seen = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1
    if world != args.gpus or ranks_seen != args.gpus:
        print(f"error: --gpus {args.gpus} but the job has WORLD_SIZE={world} "
              f"(process group: {ranks_seen} ranks)", file=sys.stderr)
        sys.exit(2)
    if args.cpu:
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", D.gpu_index(lrank))
        torch.cuda.set_device(dev)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
    rank = D.get_rank()

    cfg = get_preset(args.model, seq_len=args.seq_len)
    torch.manual_seed(args.seed)
    with torch.device(dev):
        prev = torch.get_default_dtype()
        torch.set_default_dtype(torch.bfloat16)
        model = Transformer(cfg)
        torch.set_default_dtype(prev)
    from pyrecover_amd.trainer import _use_shard_optimizer

    shard = _use_shard_optimizer(args.shard_optimizer, world, model, args.batch_per_gpu * args.seq_len,
                                 dev.type == "cuda")
    flat = model.flatten_(tokens_per_step=args.batch_per_gpu * args.seq_len, shadows=False if shard else None)
    if world > 1:
        broadcast_flat(flat)
    bucket_tune = None
    if args.bucket_mb == "auto":
        from pyrecover_amd.parallel.bucket_tune import autotune_bucket_mb

        args.bucket_mb, bucket_tune = autotune_bucket_mb(dev, flat.grad.dtype, backend=args.allreduce)
    from pyrecover_amd.trainer import _use_sparse_embedding

    sparse = _use_sparse_embedding(args.sparse_embedding_grad, world, args.batch_per_gpu * args.seq_len, cfg.vocab_size)
    reducer = GradReducer(flat, bucket_cap_mb=args.bucket_mb, backend=args.allreduce, shard=shard,
                          sparse_slot=flat.slot(model.tok_embeddings.weight).index if sparse else None)
    timer = reducer.enable_comm_timing() if world > 1 and not args.no_comm_timing else None
    opt = FlatAdamW(flat, lr=args.lr, fused=True, grad_scale=1.0 / world,
                    master_weights=args.master_weights == "fp32")
    if not args.no_overlap_optimizer:
        opt.enable_overlap(reducer)
    sched = build_lr_scheduler(opt, 10)

    B, S = args.batch_per_gpu, args.seq_len
    gen = torch.Generator(device=dev)
    gen.manual_seed(args.seed * 1000 + rank)

    def batch():
        t = torch.randint(0, cfg.vocab_size, (B, S + 1), device=dev, generator=gen)
        return t[:, :-1], t[:, 1:]

    phases = []
    sg = None
    if args.graph:
        from pyrecover_amd.graph import StepGraph, capture_allowed

        ok, why = capture_allowed(world)
        if not ok:
            print(f"error: --graph: {why}", file=sys.stderr)
            sys.exit(2)

        sg = StepGraph(model, opt, reducer)
    n_eager = [0]

    def step(timed=False):
        x, y = batch()
        if sg is not None and n_eager[0] >= 2:
            loss = sg.step(x, y)
            sched.step()
            return loss
        n_eager[0] += 1
        if timed and timer is not None:
            timer.begin_step()
        ev = ([torch.cuda.Event(enable_timing=True) for _ in range(4)]
              if timed and args.phase_timing and dev.type == "cuda" else None)
        opt.zero_grad()
        if ev:
            ev[0].record()
        loss = model(x, labels=y)
        if ev:
            ev[1].record()
        loss.backward()
        reducer.finish()
        if ev:
            ev[2].record()
        opt.step()
        sched.step()
        if ev:
            ev[3].record()
            phases.append(ev)
        return loss

    for _ in range(args.warmup):
        loss = step()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if args.profile_steps and i < args.profile_steps and dev.type == "cuda":
            torch.cuda.nvtx.range_push(f"step{i}")
        loss = step(timed=True)
        if args.profile_steps and i < args.profile_steps and dev.type == "cuda":
            torch.cuda.nvtx.range_pop()
    sync()
    if world > 1:
        torch.distributed.barrier()
    sync()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(dt_t, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt_t.item())
    final_loss = float(loss.item())
    # after the clock stopped: are the replicas still identical? (parallel/consistency.py)
    from pyrecover_amd.parallel.consistency import replica_report

    replicas = replica_report(flat, opt)
    probe = None
    if world > 1 and args.comm_probe != "off":
        # after the clock stopped: the group's all-reduce latency / bus bandwidth, measured
        from pyrecover_amd.parallel import bucket_tune as BT

        probe = {"rccl": BT._summary(BT.probe_allreduce(dev, flat.grad.dtype), world)}
        if args.comm_probe == "all" and dev.type == "cuda":
            try:
                probe["xgmi"] = BT._summary(BT.probe_xgmi(dev, flat.grad.dtype), world)
            except Exception as e:  # noqa: BLE001 - raised on every rank (XgmiAllReduce decides collectively)
                probe["xgmi"] = f"not available: {str(e).splitlines()[0][:160]}"
    tokens = B * S * world * args.steps
    tps = tokens / dt
    n_params = model.num_params()
    fpt = num_flop_per_token(model.num_params(exclude_embedding=True), cfg)
    comm = None
    if timer is not None:
        comm = timer.summary(world)
        e = torch.tensor([comm.get("exposed_comm_ms", 0.0)], device=dev, dtype=torch.float64)
        per_rank = [torch.zeros_like(e) for _ in range(world)]
        torch.distributed.all_gather(per_rank, e)
        comm["exposed_comm_ms_per_rank"] = [round(float(x.item()), 3) for x in per_rank]
    if rank == 0:
        out = {
            "metric": f"tokens/sec at seq={S} bf16 (job aggregate over all GPUs; per-GPU in tokens_per_sec_per_gpu)",
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "device": "cpu (gloo test run, not a benchmark)" if dev.type == "cpu" else "MI355X",
            "data": "synthetic (uniform random token ids), random-init weights",
            "config": {"model": f"{args.model}-shape ({n_params / 1e9:.2f}B params)", "global_batch": B * world,
                       "seq_len": S, "parallelism": f"dp{world}", "batch_per_gpu": B,
                       "bucket_mb": args.bucket_mb if world > 1 else None,
                       "bucket_autotune": bucket_tune,
                       "master_weights": args.master_weights,
                       "shard_optimizer": shard,
                       "sparse_embedding_grad": bool(sparse and world > 1),
                       "allreduce": (None if world == 1 else "xgmi" if args.allreduce == "xgmi" else
                                     "rccl" if torch.distributed.get_backend() == "nccl" else
                                     torch.distributed.get_backend()),
                       "dist_backend": torch.distributed.get_backend() if world > 1 else None,
                       "grad_buckets": reducer.num_buckets,
                       "rccl_high_priority_stream": os.environ.get("PYRECOVER_RCCL_HIGH_PRIORITY", "1") == "1",
                       "optimizer": "AdamW (flat fused HIP)" + ("" if args.no_overlap_optimizer else
                                                                 f", overlapped with backward ({_opt_sched(B * S)})"),
                       "adamw_math": "hw rcp/sqrt (fast)" if _adamw_fast() else "torch _fused_adamw_ bit-exact",
                       "weight_shadows": ",".join(getattr(flat, "shadow_sites", ())) or False,
                       "hand_written_gemms": _gemm_sites(B * S, cfg.dim)},
            "tokens_per_sec_per_gpu": round(tps / world, 2),
            "model_tflops_per_gpu": round(fpt * tps / world / 1e12, 2),
            "mfu_pct_vs_2.5PF": round(100 * fpt * tps / world / 2.5e15, 2),
            "final_loss": round(final_loss, 4),
            "peak_mem_gib": round(torch.cuda.max_memory_allocated(dev) / 2**30, 1) if dev.type == "cuda" else None,
            "gemm_table": bool(torch.cuda.tunable.is_enabled()) if dev.type == "cuda" else False,
            "hip_graph": bool(args.graph),
            "params_identical_across_ranks": replicas["params_identical_across_ranks"],
            "optimizer_identical_across_ranks": replicas["optimizer_identical_across_ranks"],
        }
        if replicas["mismatched"]:
            out["replica_checksums"] = {k: replicas["checksums"][k] for k in replicas["mismatched"]}
        if world > 1:
            out["comm"] = comm
            out["comm_env"] = comm_env()
            out["comm_probe"] = probe
        if phases:
            n = len(phases)
            out["phase_ms"] = {k: round(sum(e[i].elapsed_time(e[i + 1]) for e in phases) / n, 2)
                               for i, k in enumerate(("forward", "backward+reduce", "optimizer"))}
        print(json.dumps(out), flush=True)
    from pyrecover_amd.utils.gemm_tuning import flush_tuning

    if rank == 0:
        flush_tuning()
    if world > 1:
        torch.distributed.destroy_process_group()
    if replicas["mismatched"]:
        print(f"error: replicas differ across ranks after the timed steps: {replicas['mismatched']}", file=sys.stderr)
        sys.exit(3)


if __name__ == "__main__":
    main()
