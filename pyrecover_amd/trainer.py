"""Training orchestrator (``train.py``): the reference's loop (reference train.py:37-400) on the
MI355X engine.

Same control flow, log lines, CSV, checkpoint naming/frequency and time-aware stop semantics as
the reference, with these engine-level differences:

* model: fused HIP ops + flat parameter/gradient buffers (:mod:`pyrecover_amd.models.llama`);
* DDP: in-place bucketed RCCL all-reduce overlapped with backward (:mod:`.parallel.ddp`);
* optimizer: one flat AdamW kernel (:mod:`.optim.adamw`);
* data: resumable deterministic sampler whose cursor is checkpointed, tokenization
  in DataLoader workers (D19), the batch after an epoch boundary is a real new batch (D6);
* checkpoints: native engine, optionally asynchronous (snapshot fenced before the next optimizer
  step), atomic files, streaming md5;
* time-aware stop: the stop flag is only broadcast when time-aware checkpointing is on (D16),
  signal-triggered stop and SLURM resubmission are available.
"""
from __future__ import annotations

import csv
import json
import logging
import os
import random
import time
from pathlib import Path

import torch
from torch.utils.data import DataLoader

from . import resubmit as resub
from .ckpt import core as ckcore
from .ckpt.sharded import finalize_pending, load_ckpt_distributed, save_ckpt_distributed
from .ckpt.vanilla import load_ckpt_vanilla, save_ckpt_vanilla
from .cli import PRECISION_STR_TO_DTYPE, set_default_dtype
from .config import get_preset
from .data.dataset import CollatorForCLM, ParquetDataset, SyntheticTokenDataset
from .data.sampler import ResumableDistributedSampler
from .data.tokenizer import load_tokenizer
from .models.llama import Transformer
from .optim.adamw import FlatAdamW
from .optim.lr import build_lr_scheduler
from .parallel import dist as D
from .parallel.ddp import GradReducer, broadcast_flat
from .timelimit import TimeAwareStopper, get_job_end_time
from .utils.flops import num_flop_per_token
from .utils.gemm_tuning import configure_gemm_tuning

logger = logging.getLogger("pyrecover")
log_rank0 = D.log_rank0


def _set_op_ranges(on: bool):
    """Per-op roctx ranges inside the HIP extension ("pyrecover::attn_fwd", ...)."""
    from . import _ext

    if _ext.available():
        _ext.native().set_roctx(on)


def _profiler_start():
    """Profiler window (reference train.py:237-239): hip profiler start + per-op roctx ranges."""
    try:
        torch.cuda.cudart().cudaProfilerStart()
    except Exception:  # pragma: no cover
        pass
    _set_op_ranges(True)


def _profiler_stop():
    _set_op_ranges(False)
    try:
        torch.cuda.cudart().cudaProfilerStop()
    except Exception:  # pragma: no cover
        pass


class _StepTimer:
    """Device-side step durations from events recorded at each step end (polled, never blocking).

    The time-aware stop takes its iteration time from here, not from the host: the host runs
    ahead of the GPU, so the host span of an ordinary step under-counts, and the span of a step
    that synchronised (the log step's ``.item()``, the CSV) counts the drain of every queued
    step. ``record()`` returns the longest step completed since the last call. ``gap()`` marks a
    host-side pause that is not training time (a checkpoint save): the interval spanning it is
    dropped. ``window()`` returns (mean, max, count) of the steps completed since the last
    ``window()`` (the JSONL log)."""

    def __init__(self, enabled: bool):
        self.enabled = enabled
        self.events = []  # (event, measure_from_previous)
        self.last = None
        self._skip_next = False
        self._win = []

    def gap(self):
        self._skip_next = True

    def record(self) -> float:
        if not self.enabled:
            return 0.0
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.events.append((ev, not self._skip_next))
        self._skip_next = False
        longest = 0.0
        while self.events and self.events[0][0].query():
            e, measure = self.events.pop(0)
            if self.last is not None and measure:
                dt = self.last.elapsed_time(e) / 1000.0
                longest = max(longest, dt)
                self._win.append(dt)
            self.last = e
        return longest

    def window(self):
        w, self._win = self._win, []
        if not w:
            return None, None, 0
        return sum(w) / len(w), max(w), len(w)


class _StopFlagSync:
    """Rank 0's stop decision broadcast to every rank without a per-step host sync.

    The reference broadcasts ``should_stop`` and calls ``.item()`` at the end of every step
    (train.py:343-346), which drains the device queue each step. Here the
    broadcast of step t is enqueued asynchronously, its result is copied into pinned host memory
    behind an event, and it is read at the end of step t+1: every rank acts on the same broadcast,
    one step later, and the host keeps one step of run-ahead. The time-aware threshold budgets
    6 iterations (reference train.py:304), so the extra step fits."""

    def __init__(self, device: torch.device):
        self.cuda = device.type == "cuda"
        self.dev = torch.zeros(1, dtype=torch.int32, device=device)
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=self.cuda)
        self.pending = None

    def collect(self) -> bool:
        """Result of the previously posted broadcast (False when none is pending)."""
        if self.pending is None:
            return False
        work, ev = self.pending
        self.pending = None
        if ev is not None:
            ev.synchronize()
            return bool(self.host[0])
        work.wait()
        return bool(self.dev[0])

    def post(self, flag: bool) -> bool:
        """Collect the previous step's decision, then broadcast this step's; returns the former."""
        prev = self.collect()
        self.dev.fill_(1 if flag else 0)
        work = torch.distributed.broadcast(self.dev, src=0, async_op=True)
        ev = None
        if self.cuda:
            work.wait()  # the current stream waits for the collective; the host does not
            self.host.copy_(self.dev, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self.pending = (work, ev)
        return prev


def train(args):
    training_start_time = time.perf_counter()
    total_checkpoint_store_time = 0.0
    total_checkpoint_load_time = 0.0

    local_rank, world_size = D.maybe_init_distributed(args.distributed)
    rank = D.get_rank()
    is_dist = world_size > 1
    log_rank0(f"Experiment args: {args}")
    use_cuda = torch.cuda.is_available()
    device = torch.device("cuda", D.gpu_index(local_rank)) if use_cuda else torch.device("cpu")
    model_dtype = PRECISION_STR_TO_DTYPE[args.model_dtype]
    torch.manual_seed(args.seed)
    random.seed(args.seed)
    configure_gemm_tuning(getattr(args, "gemm_tuning", "auto"))

    # ---------------- data (reference train.py:53-84) ----------------
    log_rank0("Setting up DataLoaders...")
    seq_len = args.sequence_length
    global_batch_size = int(args.batch_size)
    local_batch_size = max(global_batch_size // world_size, 1)
    accum = max(1, int(getattr(args, "grad_accumulation_steps", 1) or 1))
    n_samples = args.batch_size * args.training_steps * accum
    preset = get_preset(args.model_preset)
    if args.synthetic_data:
        vocab = args.vocab_size or preset.vocab_size
        pad_id = 0
        train_ds = SyntheticTokenDataset(vocab, seq_len, n_samples, seed=args.seed, pad_token_id=pad_id)
    else:
        tokenizer = load_tokenizer(args.tokenizer_name_or_path)
        train_ds = ParquetDataset(args.dataset, tokenizer, seq_len, n_samples)
        vocab = args.vocab_size or tokenizer.vocab_size
        pad_id = tokenizer.pad_token_id
    log_rank0(f"Global batch size: {global_batch_size}\nLocal batch size: {local_batch_size}")
    if local_batch_size * world_size != global_batch_size:
        # reference train.py:62-63 keeps max(B//W,1) per rank but counts B·S tokens per step
        # (:252); here throughput counts what actually runs
        log_rank0(f"Note: --batch-size {global_batch_size} is not a multiple of world size {world_size}: "
                  f"each step runs {local_batch_size} x {world_size} = {local_batch_size * world_size} "
                  f"sequences, and tokens/s counts those")
    if accum > 1:
        log_rank0(f"Gradient accumulation: {accum} micro-batches per step "
                  f"({global_batch_size * accum} sequences per optimizer step)")
    train_sampler = ResumableDistributedSampler(len(train_ds), num_replicas=world_size, rank=rank, shuffle=True,
                                                seed=args.seed)
    train_collator = CollatorForCLM(seq_len, pad_id)
    train_dl = DataLoader(train_ds, batch_size=local_batch_size, collate_fn=train_collator, sampler=train_sampler,
                          num_workers=args.num_workers, pin_memory=use_cuda,
                          persistent_workers=False)

    # ---------------- model / parallelism / optimizer ----------------
    log_rank0(f"Setting up Model ({args.model_preset})...")
    model_config = get_preset(args.model_preset, seq_len=seq_len, vocab_size=vocab, n_layers=args.n_layers,
                              use_flash_attention=args.use_flash_attention)
    with set_default_dtype(model_dtype), torch.device(device):
        model = Transformer(model_config)
    model.activation_checkpointing = bool(getattr(args, "activation_checkpointing", False))
    shard = _use_shard_optimizer(getattr(args, "shard_optimizer", "off"), world_size if is_dist else 1, model,
                                 local_batch_size * seq_len,
                                 device.type == "cuda" and model_dtype in (torch.bfloat16, torch.float16))
    # the sharded optimizer's owned chunks cut matrices: no transposed weight shadows (each would be
    # re-derived from the gathered parameters every step)
    flat = model.flatten_(tokens_per_step=local_batch_size * seq_len, shadows=False if shard else None)
    overlap = not (args.clip_grad or args.no_overlap_optimizer)
    reducer = None
    if is_dist:
        broadcast_flat(flat)
    bucket_mb = args.bucket_cap_mb
    if bucket_mb == "auto" and is_dist and args.resume_from_checkpoint is not None:
        # a resumed run keeps the bucket layout it was checkpointed with: bucket boundaries decide
        # how every element's contributions are summed (bit-exact resume)
        saved = ckcore.peek_reduction(args.resume_from_checkpoint, exp_dir=Path(args.checkpoint_dir) /
                                      args.experiment_name, distributed=args.use_torch_distributed_ckpt)
        if saved and saved.get("bucket_mb"):
            bucket_mb = float(saved["bucket_mb"])
            log_rank0(f"Bucket size {bucket_mb} MiB from the checkpoint (--bucket-cap-mb auto, resume)")
    if bucket_mb == "auto":
        from .parallel.bucket_tune import autotune_bucket_mb

        bucket_mb, tune = (autotune_bucket_mb(device, flat.grad.dtype, backend=args.allreduce, flat=flat)
                           if is_dist else (256.0, {"world": 1}))
        log_rank0(f"Bucket autotune: {bucket_mb} MiB {tune}")
    sparse_emb = _use_sparse_embedding(getattr(args, "sparse_embedding_grad", "off"), world_size,
                                       local_batch_size * seq_len * accum, vocab)
    if is_dist or overlap:
        reducer = GradReducer(flat, bucket_cap_mb=bucket_mb, backend=args.allreduce, shard=shard,
                              sparse_slot=flat.slot(model.tok_embeddings.weight).index if sparse_emb else None)
        log_rank0(f"Gradient buckets: {reducer.num_buckets}, {sum(reducer.bucket_bytes()) / 2**30:.2f} GiB"
                  f"{(' (RCCL reduce-scatter + all-gather, sharded optimizer)' if shard else ' (RCCL all-reduce)') if is_dist else ''}"
                  f"{', sparse embedding-gradient exchange' if sparse_emb and is_dist else ''}")
        if reducer.force_collective and not is_dist:
            log_rank0("Bucket collectives forced on in a 1-rank "
                      f"{torch.distributed.get_backend()} group (PYRECOVER_FORCE_ALLREDUCE=1)")
    D.set_reducer_settings(bucket_mb=float(bucket_mb) if is_dist else None, allreduce=args.allreduce if is_dist else None,
                           shard_optimizer=shard, sparse_embedding=bool(sparse_emb and is_dist))
    model.train()
    # SUM all-reduce of `accum` summed micro-batch gradients: the mean is folded into the update
    grad_scale = 1.0 / (world_size * accum)
    optimizer = FlatAdamW(flat, lr=args.learning_rate, fused=args.fused_optimizer, grad_scale=grad_scale,
                          master_weights=getattr(args, "master_weights", "none") == "fp32")
    if optimizer.master is not None:
        log_rank0(f"fp32 master weights: {optimizer.master.numel() * 4 / 2**30:.2f} GiB "
                  f"(+ fp32 moments {2 * optimizer.exp_avg.numel() * 4 / 2**30:.2f} GiB)")
    if overlap:
        optimizer.enable_overlap(reducer)
        optimizer.pre_update_fences.append(ckcore.fence_all)
    lr_scheduler = build_lr_scheduler(optimizer, args.lr_warmup_steps)
    step_graph = None
    if args.compile and accum > 1:
        log_rank0("--compile with --grad-accumulation-steps > 1: running eagerly")
    elif args.compile:
        from .graph import capture_allowed

        cap_ok, cap_why = capture_allowed(world_size)
        if cap_ok and (shard or (sparse_emb and is_dist)):  # host-side bookkeeping between collectives
            cap_ok, cap_why = False, "the sharded optimizer / sparse embedding exchange are not captured"
        if not cap_ok:
            log_rank0(f"--compile: running eagerly: {cap_why}")
        elif use_cuda:
            from .graph import StepGraph

            pre = (lambda: setattr(optimizer, "grad_scale_dev",
                                   _clip_coef(flat, args.grad_max_norm, grad_scale, reducer))) if args.clip_grad else None
            step_graph = StepGraph(model, optimizer, reducer, fences=[ckcore.fence_all], pre_step=pre)
            log_rank0(f"--compile: the training step is captured into a HIP graph after "
                      f"{args.compile_warmup_steps} eager steps and replayed (no Inductor/Triton)")
        else:
            log_rank0("--compile: no GPU, running eagerly")
    eager_steps_this_run = 0
    step_timer = _StepTimer(use_cuda)
    # per-bucket collective timing for the JSONL (events only, no sync inside the step)
    comm_timer = reducer.enable_comm_timing() if (is_dist and reducer is not None and args.metrics_jsonl) else None
    ckpt_window = []  # host stall of each save issued since the last log line
    if args.async_checkpoint and int(args.checkpoint_frequency) > 0 and use_cuda:
        # params + AdamW moments (+ slack for the small entries); sharded saves need ~1/W of it.
        # Allocated now, while the GPU is idle: hipHostMalloc maps the pool into the GPU's page
        # tables, and doing that under running kernels (a background thread during the first
        # steps) was measured at 150 s for 11 GB instead of ~2 s.
        est = optimizer.checkpoint_bytes() // (world_size if args.use_torch_distributed_ckpt else 1)
        t0 = time.perf_counter()
        ckcore.Checkpointer.get(device).prewarm(int(est * 1.05) + (64 << 20), background=False)
        log_rank0(f"Pinned checkpoint staging pool: {est / 2**30:.2f} GiB in {time.perf_counter() - t0:.2f}s")
    num_flop_per_token_ = num_flop_per_token(model.num_params(exclude_embedding=True), model_config)
    log_rank0(f"Model parameters: {model.num_params() / 1e9:.3f} B, FLOPs/token: {num_flop_per_token_ / 1e9:.2f} G")

    ntokens_since_last_log = 0
    ntraining_tokens_since_last_log = 0
    time_last_log = time.perf_counter()

    # ---------------- checkpoint dirs / CSV (reference train.py:135-161) ----------------
    checkpoint_freq_steps = int(args.checkpoint_frequency)
    ckpt_path = Path(args.checkpoint_dir)
    if ckpt_path.exists() and not ckpt_path.is_dir():
        raise SystemExit(f"Checkpoint dir {ckpt_path} exists as file already! Abort!")
    exp_ckpt_path = ckpt_path / args.experiment_name
    exp_ckpt_path.mkdir(parents=True, exist_ok=True)
    csv_file = csv_writer = None
    if args.log_loss_to_csv and D.is_rank0():
        csv_path = exp_ckpt_path / f"{args.experiment_name}_loss_log.csv"
        resume_csv = args.resume_from_checkpoint is not None and csv_path.exists()
        csv_file = open(csv_path, "a" if resume_csv else "w", newline="")
        csv_writer = csv.writer(csv_file)
        if not resume_csv:
            csv_writer.writerow(["Step", "Loss"])
        csv_file.flush()
    metrics_f = open(args.metrics_jsonl, "a") if (args.metrics_jsonl and D.is_rank0()) else None
    if args.use_torch_distributed_ckpt:
        log_rank0("Using sharded (torch.distributed.checkpoint-compatible) checkpointing")
        save_ckpt_fn, load_ckpt_fn = save_ckpt_distributed, load_ckpt_distributed
    else:
        log_rank0("Using vanilla checkpointing")
        save_ckpt_fn, load_ckpt_fn = save_ckpt_vanilla, load_ckpt_vanilla

    def ckpt_name(step, final=False):
        suffix = "_final" if final else ""
        return exp_ckpt_path / (f"ckpt_{step}{suffix}" if args.use_torch_distributed_ckpt else f"ckpt_{step}{suffix}.pt")

    def do_save(step, epoch, final=False):
        p = ckpt_name(step, final)
        t0 = time.perf_counter()
        kw = {}
        if final and not args.use_torch_distributed_ckpt:
            # the final (time-aware) checkpoint computes its whole-file .md5 inline, so the sidecar
            # the reference's verified load requires (pyrecover/checkpoint.py:157-175) exists when
            # the save returns; the stop threshold budgets that digest (SaveCostModel)
            kw["defer_md5"] = False
        save_ckpt_fn(model, optimizer, lr_scheduler, train_sampler, step, epoch, p,
                     max_keep=args.max_kept_checkpoints, verify=args.verify_checkpoints, is_distributed=is_dist,
                     rank=rank, async_save=(args.async_checkpoint and not final), fsync=not args.no_fsync, **kw)
        if final:
            ckcore.wait_all()
            if args.use_torch_distributed_ckpt:
                finalize_pending()
        return p, time.perf_counter() - t0

    # ---------------- time-aware (reference train.py:163-190) ----------------
    stopper = None
    if args.timeaware_checkpointing:
        stopper = TimeAwareStopper(args.default_iter_time, args.default_ckpt_time, end_time=get_job_end_time(),
                                   install_signals=args.handle_signals)
        log_rank0(f"Initial max_iter_time: {stopper.max_iter}, max_ckpt_time: {stopper.max_ckpt}, "
                  f"buffer_time: {stopper.buffer}")
        if stopper.end_time is None:
            log_rank0("Warning: SLURM_JOB_END_TIME is not set. Time-check logic will be skipped.")
        log_rank0(f"SLURM_JOB_END_TIME: {stopper.end_time}")
    cost = None
    if stopper is not None:
        if is_dist:
            stopper.extra_iters = 1  # every rank acts on rank 0's decision one step later (_StopFlagSync)
        # what the final save writes on this rank: params + AdamW m, v (+ the fp32 master with
        # --master-weights fp32: 14 instead of 6 B/param) (+ small entries)
        state_bytes = optimizer.checkpoint_bytes()
        if args.use_torch_distributed_ckpt:
            state_bytes = -(-state_bytes // world_size)
        inline_md5 = bool(args.verify_checkpoints) and not args.use_torch_distributed_ckpt
        cost = ckcore.SaveCostModel(state_bytes, inline_md5)
        if D.is_rank0() or args.use_torch_distributed_ckpt:
            t0 = time.perf_counter()
            try:
                cost.probe(exp_ckpt_path)
            except Exception as e:  # noqa: BLE001 - an unprobeable directory: the prior stays
                log_rank0(f"Save-cost probe failed ({e}); budgeting the final save from --default-ckpt-time")
            stopper.set_ckpt_estimate(cost.final_seconds())
            log_rank0(f"Save-cost probe ({time.perf_counter() - t0:.2f}s): write {cost.write_bps / 1e9:.2f} GB/s"
                      + (f", serial MD5 {cost.md5_bps / 1e9:.2f} GB/s" if inline_md5 else "")
                      + f"; final checkpoint of {state_bytes / 2**30:.2f} GiB estimated at "
                      f"{stopper.ckpt_estimate:.2f}s (budget {stopper.ckpt_budget:.2f}s, threshold "
                      f"{stopper.threshold:.2f}s)")
    if args.resubmit != "none":
        resub.setup_resubmission(args.resubmit, args.resubmit_script,
                                 [a for a in os.environ.get("PYRECOVER_SCRIPT_ARGS", "").split() if a],
                                 max_resubmits=args.max_resubmits)

    # ---------------- resume (reference train.py:192-212) ----------------
    train_step = 0
    epoch = 1
    train_sampler.set_epoch(epoch)
    if args.resume_from_checkpoint is not None:
        log_rank0(f"Try resume from checkpoint {args.resume_from_checkpoint}")
        t0 = time.perf_counter()
        epoch, train_step = load_ckpt_fn(model, optimizer, lr_scheduler, train_sampler, args.resume_from_checkpoint,
                                         experiment_dir=exp_ckpt_path, verify=args.verify_checkpoints,
                                         is_distributed=is_dist, rank=rank)
        epoch = epoch or 1
        dt = time.perf_counter() - t0
        total_checkpoint_load_time += dt
        log_rank0(f"Checkpoint loading completed in {dt:.2f} seconds")
    D.barrier()

    # cross-rank replica check (parallel/consistency.py): every N steps and at the end
    check_every = args.replica_check_every if getattr(args, "replica_check_every", None) is not None \
        else 10 * max(1, int(args.logging_frequency))
    train_dl_iterator = iter(train_dl)
    should_stop = False
    local_stop = False  # rank 0's own time decision (latched; acted on via the broadcast when W > 1)
    stopped_for_time = False
    stop_sync = _StopFlagSync(device) if (stopper is not None and is_dist) else None
    log_rank0("Starting training!")
    if world_size > 1:
        print(f"[Rank {rank}] Starting training on {device}", flush=True)
    loss = None
    while train_step < args.training_steps:
        train_step += 1
        if cost is not None:
            # async saves stall training for ~ms, but the final save is synchronous, first drains
            # the in-flight write, and (with --verify-checkpoints) computes the serial whole-file
            # MD5 inline: budget it from bytes and measured rates
            ckcore.poll_all()
            if stopper.set_ckpt_estimate(cost.final_seconds()):
                log_rank0(f"Updated final checkpoint estimate from measured rates: {stopper.ckpt_estimate:.2f}s")
            stopper.inflight_drain = cost.drain_seconds(stopper.ckpt_budget)
        if stopper is not None and D.is_rank0() and not local_stop and stopper.should_stop():
            local_stop = True
            rem = stopper.remaining()
            log_rank0(f"[TIME CHECK] Remaining time ({rem if rem is not None else float('nan'):.2f}s) < threshold "
                      f"({stopper.threshold:.2f}s = {1 + stopper.extra_iters} x iter {stopper.max_iter:.2f}s + ckpt "
                      f"{stopper.ckpt_budget:.2f}s + buffer {stopper.buffer:.2f}s + in-flight drain "
                      f"{stopper.inflight_drain:.2f}s). should_stop set to True.")
        iter_start = time.perf_counter()
        if args.profile and args.profile_step_start == train_step:
            _profiler_start()
        if args.profile and args.profile_step_start <= train_step <= args.profile_step_end:
            torch.cuda.nvtx.range_push(f"step_{train_step}") if use_cuda else None

        micro = []
        for _ in range(accum):
            train_sampler.set_epoch(epoch)
            try:
                input_ids, labels = next(train_dl_iterator)
            except StopIteration:
                epoch += 1
                train_sampler.set_epoch(epoch)
                train_dl_iterator = iter(train_dl)
                input_ids, labels = next(train_dl_iterator)
            train_sampler.advance(input_ids.shape[0])

            # true tokens of this step on all ranks (every rank runs the same local batch)
            ntokens_since_last_log += input_ids.shape[0] * world_size * seq_len
            num_items_in_batch = labels.ne(-100).sum()
            ntraining_tokens_since_last_log += int(num_items_in_batch) * world_size
            micro.append((input_ids.to(device, non_blocking=True), labels.to(device, non_blocking=True)))

        if step_graph is not None and eager_steps_this_run >= args.compile_warmup_steps:
            loss = step_graph.step(*micro[0])  # fences the snapshot before the replay
        else:
            if comm_timer is not None:
                comm_timer.begin_step()
            optimizer.zero_grad()
            loss = None
            for m, (input_ids, labels) in enumerate(micro):
                if m:
                    flat.next_micro_batch()  # producers now add into the written gradients
                if reducer is not None:
                    # no communication (or overlapped update) until the last micro-batch
                    reducer.enabled = m == accum - 1
                lm = model(input_ids, labels=labels)
                lm.backward()
                loss = lm.detach() if loss is None else loss + lm.detach()
            if accum > 1:
                loss = loss / accum
            if reducer is not None:
                reducer.finish()
            if args.clip_grad:
                optimizer.grad_scale_dev = _clip_coef(flat, args.grad_max_norm, grad_scale, reducer)
            ckcore.fence_all()  # an async snapshot must land before parameters change
            optimizer.step()
            eager_steps_this_run += 1
        lr_scheduler.step()

        if csv_writer is not None:
            csv_writer.writerow([train_step, loss.item()])
            csv_file.flush()

        if train_step == 1 or train_step % args.logging_frequency == 0:
            # sync first: the host runs ahead of the GPU, so an unsynchronized clock would count
            # queued-but-unexecuted steps (the reference reads the clock before its .item())
            lval = loss.item()
            time_delta = time.perf_counter() - time_last_log
            tps = ntokens_since_last_log / time_delta
            per_gpu = tps / world_size
            mfu = 100 * num_flop_per_token_ * per_gpu / (args.peak_tflops * 1e12)
            tflops = num_flop_per_token_ * per_gpu / 1e12
            training_tps = ntraining_tokens_since_last_log / time_delta
            log_rank0(f"Epoch: {epoch} | Step: {train_step} | Loss: {lval:.2f} | Tokens per second: {tps:.2f} | "
                      f"Training tokens per second (%): {100 * training_tps / tps:.2f} | MFU (%): {mfu:.2f} | "
                      f"TFLOPs: {tflops:.2f} | Tokens per second per GPU: {per_gpu:.2f}")
            if metrics_f is not None:
                rec = {"step": train_step, "epoch": epoch, "loss": lval, "tokens_per_s": tps,
                       "tokens_per_s_per_gpu": per_gpu, "mfu_pct": mfu, "tflops_per_gpu": tflops,
                       "time": time.time()}
                rec.update(_diagnostics(step_timer, device, comm_timer, world_size, ckpt_window, stopper))
                metrics_f.write(json.dumps(rec) + "\n")
                metrics_f.flush()
            elif comm_timer is not None:
                comm_timer.steps.clear()
            ckpt_window.clear()
            ntokens_since_last_log = 0
            ntraining_tokens_since_last_log = 0
            time_last_log = time.perf_counter()

        if is_dist and check_every > 0 and train_step % check_every == 0:
            _replica_check(flat, optimizer, train_step)

        dev_step = step_timer.record()
        if stopper is not None:
            # GPU: device time per step from events (no sync; never the host span, which
            # under-counts while the host runs ahead and counts the drain of every queued step on
            # a step that synchronised for logging). CPU: the host span (synchronous execution).
            iter_time = dev_step if use_cuda else time.perf_counter() - iter_start
            if stopper.update_iter(iter_time):
                log_rank0(f"Updated max_iter_time: {stopper.max_iter}")
            if train_step % args.logging_frequency == 0:
                log_rank0(f"Current buffer_time: {stopper.buffer}")

        if checkpoint_freq_steps > 0 and train_step % checkpoint_freq_steps == 0:  # 0 or -1: off
            log_rank0(f"Saving checkpoint to {ckpt_name(train_step)}")
            _, store_time = do_save(train_step, epoch)
            step_timer.gap()
            ckpt_window.append(store_time)
            total_checkpoint_store_time += store_time
            if stopper is not None and stopper.update_ckpt(store_time):
                log_rank0(f"Updated max_ckpt_time: {stopper.max_ckpt}")
            log_rank0(f"Checkpoint store completed in {store_time:.2f} seconds")

        if stopper is not None and is_dist:
            # rank 0's decision of the previous step (no per-step host sync)
            should_stop = stop_sync.post(local_stop or stopper.signaled)
        elif stopper is not None:
            should_stop = local_stop or stopper.signaled

        if getattr(args, "stop_at_step", None) is not None and train_step == args.stop_at_step:
            should_stop = True
            if stopper is None:
                stopper = TimeAwareStopper(args.default_iter_time, args.default_ckpt_time, end_time=None)
        if stopper is not None and should_stop:
            log_rank0(f"[TIME CHECK] Saving final checkpoint to {ckpt_name(train_step, True)} before exit.")
            final_path, store_time = do_save(train_step, epoch, final=True)
            total_checkpoint_store_time += store_time
            rem = stopper.remaining()
            log_rank0(f"[TIME CHECK] Final checkpoint store completed in {store_time:.2f} seconds (estimated "
                      f"{stopper.ckpt_estimate:.2f}s; {rem if rem is not None else float('nan'):.2f}s left)")
            stopped_for_time = True
            if args.resubmit != "none":
                resub.maybe_resubmit(rank)
            break

        if args.profile and args.profile_step_start <= train_step <= args.profile_step_end and use_cuda:
            torch.cuda.nvtx.range_pop()
        if args.profile and args.profile_step_end == train_step:
            _profiler_stop()

    # drain background checkpoint writes (and deferred .md5 digests) before reporting; after a
    # time-aware stop the digests get only the time left before the wall-clock limit (minus a
    # margin; 60 s after a signal) -- a checkpoint of this job whose digest was cut short has no
    # .md5; with --verify-checkpoints it is removed below (the final checkpoint supersedes it)
    if stop_sync is not None:
        stop_sync.collect()  # retire the last posted broadcast before teardown
    t0 = time.perf_counter()
    ckcore.wait_all()
    finalize_pending()
    if stopped_for_time:
        end = getattr(stopper, "end_time", None)
        deadline = max((end - 10.0) if end else time.time() + 60.0, time.time() + 2.0)
        if not ckcore.flush_all(deadline=deadline):
            log_rank0("[TIME CHECK] deferred .md5 digest abandoned at the wall-clock limit")
            if args.verify_checkpoints and not args.use_torch_distributed_ckpt and D.is_rank0():
                # every checkpoint kept under --verify-checkpoints carries its .md5
                for f in ckcore.drop_unverified(exp_ckpt_path, str(final_path)):
                    log_rank0(f"[TIME CHECK] removed {f}: its .md5 was not written before the limit "
                              f"(the final checkpoint supersedes it)")
    else:
        ckcore.flush_all()
    total_checkpoint_store_time += time.perf_counter() - t0
    if is_dist and check_every > 0 and loss is not None:
        _replica_check(flat, optimizer, train_step)
    total_training_time = time.perf_counter() - training_start_time
    if csv_file is not None:
        csv_file.close()
    if metrics_f is not None:
        metrics_f.close()
    log_rank0(f"Training completed in {total_training_time:.2f} seconds")
    log_rank0(f"Total checkpoint loading time: {total_checkpoint_load_time:.2f} seconds")
    log_rank0(f"Total checkpoint storing time: {total_checkpoint_store_time:.2f} seconds")
    log_rank0(f"Total checkpointing time: {(total_checkpoint_load_time + total_checkpoint_store_time):.2f} seconds")
    D.maybe_cleanup_distributed()
    return {"step": train_step, "epoch": epoch, "loss": float(loss.item()) if loss is not None else None,
            "stopped_early": should_stop}


_CKPT_SEEN = {"jobs": 0}


def _diagnostics(step_timer, device, comm_timer, world_size, ckpt_window, stopper) -> dict:
    """Extra JSONL fields of a log step: device step time, HBM, exposed all-reduce
    time and bus bandwidth, checkpoint stall / background write. Called right after the log
    step's sync, so reading the events here does not stall the device queue."""
    out = {}
    mean, mx, n = step_timer.window()
    out["device_step_ms"] = round(mean * 1e3, 3) if mean is not None else None
    out["device_step_max_ms"] = round(mx * 1e3, 3) if mx is not None else None
    if device.type == "cuda":
        out["hbm_gib"] = round(torch.cuda.memory_allocated(device) / 2**30, 3)
        out["hbm_peak_gib"] = round(torch.cuda.max_memory_allocated(device) / 2**30, 3)
        out["hbm_reserved_gib"] = round(torch.cuda.memory_reserved(device) / 2**30, 3)
    else:
        out["hbm_gib"] = out["hbm_peak_gib"] = out["hbm_reserved_gib"] = None
    if comm_timer is not None:
        if comm_timer.cuda:
            comm_timer.side.synchronize()  # its end events follow the collectives the step waited for
        summ = comm_timer.summary(world_size)
        comm_timer.steps.clear()
        out["exposed_comm_ms"] = summ.get("exposed_comm_ms")
        out["allreduce_busy_ms"] = summ.get("allreduce_busy_ms")
        out["allreduce_busbw_gbps"] = summ.get("allreduce_busbw_gbps")
    else:
        out["exposed_comm_ms"] = out["allreduce_busy_ms"] = out["allreduce_busbw_gbps"] = None
    out["ckpt_saves"] = len(ckpt_window)
    out["ckpt_stall_s"] = round(sum(ckpt_window), 4)
    jobs = ckcore.WRITE_STATS.get("jobs", 0)
    last = ckcore.WRITE_STATS.get("last") if jobs != _CKPT_SEEN["jobs"] else None
    _CKPT_SEEN["jobs"] = jobs
    out["ckpt_write_s"] = round(float(last["seconds"]), 4) if last else None
    out["ckpt_write_gib"] = round(float(last["bytes"]) / 2**30, 4) if last else None
    if stopper is not None:
        out["max_iter_time_s"] = round(stopper.max_iter, 4)
        out["ckpt_budget_s"] = round(stopper.ckpt_budget, 3)
        out["stop_threshold_s"] = round(stopper.threshold, 3)
    return out


def _clip_coef(flat, max_norm: float, pre_scale: float, reducer=None):
    """Device-side clip coefficient min(1, max_norm / ||g||) over the flat (reduced) gradient. With
    the sharded optimizer each rank holds only its chunks reduced: the squared norms of those (the
    shared tails counted on rank 0 only) are summed over the ranks."""
    from . import _ext

    if reducer is not None and reducer.shard:
        ranges = [(a, z) for b in range(reducer.num_buckets) for i, (a, z) in enumerate(reducer.owned(b))
                  if reducer.rank == 0 or a < reducer.ranges[b][0] + reducer.chunks[b] * reducer.world]
        parts = []
        for a, z in ranges:
            g = flat.grad[a:z]
            if _ext.hip(g):
                parts.append(_ext.native().grad_norm(g, max_norm, 1.0)[0:1].double() ** 2)
            else:
                parts.append(g.double().pow(2).sum().reshape(1))
        sq = torch.stack(parts).sum().reshape(1) if parts else torch.zeros(1, dtype=torch.float64,
                                                                           device=flat.grad.device)
        torch.distributed.all_reduce(sq, group=reducer.group)
        norm = sq.sqrt() * pre_scale
        return torch.clamp(max_norm / (norm + 1e-6), max=1.0).reshape(1).float()
    if _ext.hip(flat.grad):
        return _ext.native().grad_norm(flat.grad, max_norm, pre_scale)[1:2]
    norm = flat.grad.to(torch.promote_types(flat.grad.dtype, torch.float32)).norm() * pre_scale
    return torch.clamp(max_norm / (norm + 1e-6), max=1.0).reshape(1).float()


def _replica_check(flat, optimizer, step: int):
    """Collective: stop when the DDP replicas are no longer identical (parallel/consistency.py)."""
    from .parallel.consistency import replica_report

    rep = replica_report(flat, optimizer)
    if rep["mismatched"]:
        msg = (f"replica check at step {step}: {', '.join(rep['mismatched'])} differ across ranks: "
               + "; ".join(f"{k}: {rep['checksums'][k]}" for k in rep["mismatched"]))
        logger.error(msg)
        raise RuntimeError(msg)
    log_rank0(f"Replica check at step {step}: parameters"
              f"{'' if rep['optimizer_identical_across_ranks'] is None else ' and optimizer moments'} identical "
              f"on all ranks")


def _use_shard_optimizer(mode, world: int, model, tokens_per_rank: int, gpu16: bool) -> bool:
    """--shard-optimizer: on / off, or auto: W > 1, 16-bit parameters on the GPU, and a model that
    gets no transposed weight shadows at this batch (models/llama.py planned_shadow_sites; the
    sharded mode runs without them). Then ZeRO-1 costs the step nothing and each rank updates 1/W
    of the parameters: Llama-3-8B S2048 B1 at N = 8 predicted 0.85 -> 0.89 scaling at 300 GB/s
    with the sparse embedding exchange (profiles/r6/comm/comm_predict_8b_b1_with_update_cost.log). A bare
    ``--shard-optimizer`` (True) means on."""
    if world <= 1 or mode in (False, None, "off"):
        return False
    if mode is True or mode == "on":
        return True
    return bool(gpu16 and not model.planned_shadow_sites(tokens_per_rank))


def _use_sparse_embedding(mode: str, world: int, tokens_per_rank: int, vocab: int) -> bool:
    """--sparse-embedding-grad: on / off, or auto: W > 1 and the job's tokens per step at most half
    the vocabulary (then the exchanged rows are at most half of the dense gradient's, which the
    all-reduce would move twice)."""
    if mode == "on":
        return True
    if mode == "auto":
        return world > 1 and 2 * world * tokens_per_rank <= vocab
    return False
