"""``train.py`` command line: every flag of reference utils.py:105-261 (same spellings, types and
defaults, including the underscore forms ``--experiment_name`` / ``--use_flash_attention``), plus
new flags for the MI355X engine (model presets, synthetic data, seeding, async/sharded checkpoint
knobs, DDP bucket size, resubmission, gradient clipping)."""
from __future__ import annotations

import argparse
import logging
from contextlib import contextmanager

import torch

logger = logging.getLogger("pyrecover")

PRECISION_STR_TO_DTYPE = {"fp16": torch.float16, "bf16": torch.bfloat16, "fp32": torch.float32,
                          "fp64": torch.float64}



def _bucket_arg(v):
    from .parallel.bucket_tune import parse_bucket_arg

    return parse_bucket_arg(v)

def init_logger():
    """reference utils.py:19-27 (root logger at INFO with the same format)."""
    root = logging.getLogger()
    root.setLevel(logging.INFO)
    if not any(getattr(h, "_pyrecover", False) for h in root.handlers):
        ch = logging.StreamHandler()
        ch.setLevel(logging.INFO)
        ch.setFormatter(logging.Formatter("%(asctime)s - %(name)s - %(levelname)s - %(message)s"))
        ch._pyrecover = True
        root.addHandler(ch)


@contextmanager
def set_default_dtype(dtype: torch.dtype):
    """reference utils.py:92-102"""
    old = torch.get_default_dtype()
    torch.set_default_dtype(dtype)
    try:
        yield
    finally:
        torch.set_default_dtype(old)


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="pyrecover_amd training (MI355X-native DDP + checkpointing)")
    # ---- reference flags (reference utils.py:107-258) ----
    p.add_argument("--dataset", type=str, default="/capstor/store/cscs/ethz/large-sc/datasets/train_data.parquet",
                   help="Path to a parquet file containing a 'text' column with documents (`str`)")
    p.add_argument("--tokenizer-name-or-path", type=str, default="unsloth/Mistral-Nemo-Base-2407-bnb-4bit")
    p.add_argument("--sequence-length", type=int, default=2048)
    p.add_argument("--batch-size", type=int, default=1,
                   help="GLOBAL batch size; each rank uses max(batch_size // world_size, 1) (reference semantics)")
    p.add_argument("--fused-optimizer", action="store_true")
    p.add_argument("--master-weights", choices=["none", "fp32"], default="none",
                   help="fp32: AdamW updates an fp32 master copy with fp32 moments and the 16-bit model "
                        "parameters are the master rounded (default none: pure-dtype training, as the reference)")
    p.add_argument("--learning-rate", type=float, default=1e-5)
    p.add_argument("--lr-warmup-steps", type=int, default=10)
    p.add_argument("--training-steps", type=int, default=1000)
    p.add_argument("--logging-frequency", type=int, default=5)
    p.add_argument("--profile", action="store_true", help="roctx profiler window (use with rocprofv3 --selected-regions)")
    p.add_argument("--profile-step-start", type=int, default=10)
    p.add_argument("--profile-step-end", type=int, default=12)
    p.add_argument("--grad-max-norm", type=float, default=1, help="used only with --clip-grad (reference: unused)")
    p.add_argument("--model-dtype", type=str, default="bf16", choices=sorted(PRECISION_STR_TO_DTYPE))
    p.add_argument("--compile", action="store_true",
                   help="capture the whole training step into a HIP graph and replay it (the reference's "
                        "torch.compile flag; no Triton/Inductor)")
    p.add_argument("--compile-warmup-steps", type=int, default=2,
                   help="eager steps before the step graph is captured (--compile)")
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--checkpoint-dir", type=str, default="checkpoints/")
    p.add_argument("--checkpoint-frequency", type=int, default=10)
    p.add_argument("--resume-from-checkpoint", type=str, default=None)
    p.add_argument("--experiment_name", "--experiment-name", dest="experiment_name", type=str, default="default-exp")
    p.add_argument("--verify-checkpoints", action="store_true")
    p.add_argument("--max-kept-checkpoints", type=int, default=3)
    p.add_argument("--use-torch-distributed-ckpt", action="store_true",
                   help="sharded checkpoint directories (dcp-compatible layout, native writer)")
    p.add_argument("--default-iter-time", type=float, default=1.0)
    p.add_argument("--default-ckpt-time", type=float, default=10.0)
    p.add_argument("--timeaware-checkpointing", action="store_true")
    p.add_argument("--use_flash_attention", "--use-flash-attention", dest="use_flash_attention",
                   action="store_true", help="accepted for parity: the HIP flash-attention kernel is always used on GPU")
    p.add_argument("--log-loss-to-csv", action="store_true")
    # ---- new flags ----
    p.add_argument("--model-preset", type=str, default="llama3-8b",
                   help="llama3-8b (reference default architecture), llama2-7b, gpt2-medium, gpt2-small, llama-tiny")
    p.add_argument("--n-layers", type=int, default=None, help="override the preset's layer count")
    p.add_argument("--vocab-size", type=int, default=None, help="override vocab (default: tokenizer/preset)")
    p.add_argument("--synthetic-data", action="store_true", help="deterministic random tokens instead of parquet")
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--num-workers", type=int, default=2, help="DataLoader workers (tokenization off the hot loop)")
    p.add_argument("--bucket-cap-mb", type=_bucket_arg, default=256.0,
                   help="DDP all-reduce bucket size in MiB, or 'auto': probe the job's all-reduce latency and "
                        "bandwidth at startup and pick the size (parallel/bucket_tune.py)")
    p.add_argument("--allreduce", choices=["rccl", "xgmi"], default="rccl",
                   help="gradient all-reduce backend: RCCL rings (default) or the direct per-link xGMI "
                        "reduce-scatter/all-gather over IPC-mapped peer buffers (single node)")
    p.add_argument("--shard-optimizer", nargs="?", const="on", default="auto", choices=["auto", "on", "off"],
                   help="ZeRO-1 data parallelism: reduce-scatter each gradient bucket, update only this rank's "
                        "1/W of the parameters, all-gather them (replicated parameters, unchanged checkpoints); "
                        "auto: at W > 1 for 16-bit GPU models that carry no transposed weight shadows at this "
                        "batch (e.g. Llama-3-8B S2048 B1); a bare flag means on")
    p.add_argument("--sparse-embedding-grad", choices=["auto", "on", "off"], default="auto",
                   help="reduce the token-embedding gradient as (token id, row) pairs instead of a dense "
                        "all-reduce; auto: when the ranks' tokens per step are at most half the vocabulary")
    p.add_argument("--replica-check-every", type=int, default=None,
                   help="W > 1: compare a checksum of the parameters (and optimizer moments) across ranks every "
                        "N steps and at the end, and stop on a mismatch (default 10 x --logging-frequency; 0 = off)")
    p.add_argument("--async-checkpoint", action="store_true",
                   help="snapshot to pinned host memory and write in the background while training continues")
    p.add_argument("--no-fsync", action="store_true", help="skip fsync of checkpoint files")
    p.add_argument("--clip-grad", action="store_true", help="enable gradient clipping at --grad-max-norm")
    p.add_argument("--no-overlap-optimizer", action="store_true",
                   help="run AdamW after backward instead of per gradient bucket during backward")
    p.add_argument("--resubmit", choices=["none", "requeue", "chain"], default="none",
                   help="after a time-aware final checkpoint, requeue/chain the SLURM job")
    p.add_argument("--resubmit-script", type=str, default=None)
    p.add_argument("--max-resubmits", type=int, default=10,
                   help="stop resubmitting after this many requeues (SLURM_RESTART_COUNT) / chained jobs")
    p.add_argument("--handle-signals", action="store_true",
                   help="SIGUSR1/SIGTERM trigger the time-aware final checkpoint (#SBATCH --signal=B:USR1@T)")
    p.add_argument("--stop-at-step", type=int, default=None,
                   help="simulate a preemption: write the final checkpoint at this step and exit (testing)")
    p.add_argument("--metrics-jsonl", type=str, default=None, help="append per-log-step metrics as JSON lines")
    p.add_argument("--grad-accumulation-steps", type=int, default=1,
                   help="micro-batches of the local batch per optimizer step (gradients summed in place; "
                        "the all-reduce and the update run once, after the last micro-batch)")
    p.add_argument("--activation-checkpointing", action="store_true",
                   help="recompute each transformer block's forward during backward (saves activations)")
    p.add_argument("--gemm-tuning", choices=["auto", "off", "tune"], default="auto")
    p.add_argument("--peak-tflops", type=float, default=2500.0, help="MFU denominator (MI355X dense bf16)")
    return p


def get_args(argv=None):
    return build_parser().parse_args(argv)
