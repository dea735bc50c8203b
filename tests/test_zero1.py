"""Sharded optimizer (--shard-optimizer, ZeRO-1), sparse embedding-gradient exchange, cross-rank
replica checks and reduction-settings recording: multi-process gloo tests on the CPU."""
import os

import pytest
import torch
import torch.multiprocessing as mp

from tests.test_distributed import _argv, _free_port, _run


def _state(path):
    return torch.load(path, weights_only=True)


def _assert_same_state(a, b):
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    sa, sb = a["optimizer"]["state"], b["optimizer"]["state"]
    assert sorted(sa) == sorted(sb)
    for i in sa:
        for k in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[i][k], sb[i][k]), (i, k)
        assert float(sa[i]["step"]) == float(sb[i]["step"])


def _zargv(ckdir, steps, extra=()):
    # bf16 (the production dtype: every reduction rounds), small buckets so that a bucket holds
    # several slots and the shared tails are exercised
    return _argv(ckdir, steps, ["--model-dtype", "bf16", "--distributed", "--replica-check-every", "5"] + list(extra))


@pytest.mark.parametrize("world", [2, 4])
def test_shard_optimizer_bitwise_equals_allreduce(tmp_path, world):
    """20 steps: parameters AND moments of the ZeRO-1 run equal the all-reduce run's bit for bit
    (the reduce-scatter sums each element in the same order as the all-reduce; the update is
    elementwise), and the replica check passes every 5 steps."""
    n = 20
    batch = ["--batch-size", str(2 * world), "--checkpoint-frequency", str(n)]
    _run(world, _zargv(tmp_path / "ar", n, batch), tmp_path)
    _run(world, _zargv(tmp_path / "zero", n, batch + ["--shard-optimizer"]), tmp_path)
    a = _state(tmp_path / "ar" / "e" / f"ckpt_{n}.pt")
    z = _state(tmp_path / "zero" / "e" / f"ckpt_{n}.pt")
    _assert_same_state(a, z)
    red = z["pyrecover_state"]["reduction"]
    assert red["shard_optimizer"] is True and red["world_size"] == world and red["bucket_mb"] == 0.05
    assert a["pyrecover_state"]["reduction"]["shard_optimizer"] is False


def test_shard_optimizer_no_overlap_and_clip(tmp_path):
    """The non-overlapped update (after backward) and gradient clipping (global norm from the owned
    chunks, all-reduced) in ZeRO-1 mode track the all-reduce run (clipping: the norm is summed in a
    different order, so to rounding)."""
    n = 6
    ex = ["--no-overlap-optimizer", "--checkpoint-frequency", str(n)]
    _run(2, _zargv(tmp_path / "ar", n, ex), tmp_path)
    _run(2, _zargv(tmp_path / "zero", n, ex + ["--shard-optimizer"]), tmp_path)
    _assert_same_state(_state(tmp_path / "ar" / "e" / f"ckpt_{n}.pt"), _state(tmp_path / "zero" / "e" / f"ckpt_{n}.pt"))
    ex = ["--clip-grad", "--grad-max-norm", "0.05", "--checkpoint-frequency", str(n)]
    _run(2, _zargv(tmp_path / "arc", n, ex), tmp_path)
    _run(2, _zargv(tmp_path / "zc", n, ex + ["--shard-optimizer"]), tmp_path)
    a, z = _state(tmp_path / "arc" / "e" / f"ckpt_{n}.pt"), _state(tmp_path / "zc" / "e" / f"ckpt_{n}.pt")
    for k in a["model"]:
        torch.testing.assert_close(a["model"][k].float(), z["model"][k].float(), rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("fmt", ["vanilla", "sharded"])
def test_shard_optimizer_checkpoints_cross_resume(tmp_path, fmt):
    """A checkpoint written in ZeRO-1 mode resumes bit-exactly in the default mode and vice versa:
    (ZeRO-1 to step 3, default to 6) == (default to 3, ZeRO-1 to 6) == default to 6."""
    n = 6
    f = ["--use-torch-distributed-ckpt"] if fmt == "sharded" else []
    base = f + ["--checkpoint-frequency", "3"]
    # preempted at step 3 (--stop-at-step writes ckpt_3_final), resumed from it ("latest")
    _run(2, _zargv(tmp_path / "ref", n, base), tmp_path)
    _run(2, _zargv(tmp_path / "zd", n, base + ["--shard-optimizer", "--stop-at-step", "3"]), tmp_path)
    _run(2, _zargv(tmp_path / "zd", n, base + ["--resume-from-checkpoint", "latest"]), tmp_path)
    _run(2, _zargv(tmp_path / "dz", n, base + ["--stop-at-step", "3"]), tmp_path)
    _run(2, _zargv(tmp_path / "dz", n, base + ["--shard-optimizer", "--resume-from-checkpoint", "latest"]), tmp_path)
    if fmt == "vanilla":
        ref = _state(tmp_path / "ref" / "e" / f"ckpt_{n}.pt")
        for d in ("zd", "dz"):
            _assert_same_state(ref, _state(tmp_path / d / "e" / f"ckpt_{n}.pt"))
    else:
        from pyrecover_amd.ckpt.sharded import read_sharded_state

        ref = read_sharded_state(str(tmp_path / "ref" / "e" / f"ckpt_{n}"))
        for d in ("zd", "dz"):
            other = read_sharded_state(str(tmp_path / d / "e" / f"ckpt_{n}"))
            for k in ref["model"]:
                assert torch.equal(ref["model"][k], other["model"][k]), (d, k)
            for i, st in ref["optimizer"]["state"].items():
                for k in ("exp_avg", "exp_avg_sq"):
                    assert torch.equal(st[k], other["optimizer"]["state"][i][k]), (d, i, k)


# ---------------------------------------------------------------------------------------------
def _sparse_entry(rank, world, port, out_dir, accum):
    # run the exchange, keep its result, then compare with the rank-ordered dense reduction
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.parallel.ddp import GradReducer

    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    m = Transformer(get_preset("llama-micro", seq_len=64))
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    slot = flat.slot(m.tok_embeddings.weight)
    V = m.model_args.vocab_size

    def backward(enable_last):
        g = torch.Generator().manual_seed(100 + rank)
        flat.zero_grad()
        for a in range(accum):
            if a:
                flat.next_micro_batch()
            if red is not None:
                red.enabled = enable_last and a == accum - 1
            tok = torch.randint(0, min(V, 40), (2, 33), generator=g)
            m(tok[:, :-1], labels=tok[:, 1:]).backward()

    red = None
    backward(False)  # this rank's dense gradient, no communication
    local = slot.view.view(V, -1).clone()
    allg = [torch.empty_like(local) for _ in range(world)]
    torch.distributed.all_gather(allg, local)
    ref = allg[0].float()
    for r in range(1, world):
        ref = ref + allg[r].float()
    ref = ref.to(local.dtype)
    red = GradReducer(flat, bucket_cap_mb=0.05, sparse_slot=slot.index)
    assert red.bucket_slots[red.sparse_bucket] == [slot.index]  # a bucket of its own
    backward(True)
    red.finish()
    got = slot.view.view(V, -1).clone()
    torch.save({"equal": torch.equal(got, ref), "touched": int((ref != 0).any(1).sum()),
                "maxdiff": float((got.float() - ref.float()).abs().max())},
               os.path.join(out_dir, f"sparse_{rank}.pt"))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,accum", [(2, 1), (4, 1), (2, 2)])
def test_sparse_embedding_exchange_equals_rank_ordered_dense_sum(tmp_path, world, accum):
    """The (token id, row) exchange writes exactly the rank-ordered fp32 sum of the ranks' dense
    embedding gradients, rounded once to bf16, into every row (rows no rank touched stay zero),
    including the rows of earlier gradient-accumulation micro-batches."""
    mp.spawn(_sparse_entry, args=(world, _free_port(), str(tmp_path), accum), nprocs=world, join=True)
    for r in range(world):
        res = torch.load(os.path.join(tmp_path, f"sparse_{r}.pt"), weights_only=True)
        assert res["equal"], res
        assert res["touched"] > 10


def test_sparse_embedding_training_runs_and_resumes(tmp_path):
    """train.py --sparse-embedding-grad on (W = 2, bf16) next to the dense run: the embedding rows
    agree to bf16 rounding of the two reductions, the other parameters are unaffected beyond it, and
    the setting is recorded in the checkpoint."""
    n = 4
    ex = ["--checkpoint-frequency", str(n)]
    _run(2, _zargv(tmp_path / "dense", n, ex + ["--sparse-embedding-grad", "off"]), tmp_path)
    _run(2, _zargv(tmp_path / "sparse", n, ex + ["--sparse-embedding-grad", "on", "--shard-optimizer"]), tmp_path)
    a, s = _state(tmp_path / "dense" / "e" / f"ckpt_{n}.pt"), _state(tmp_path / "sparse" / "e" / f"ckpt_{n}.pt")
    assert s["pyrecover_state"]["reduction"]["sparse_embedding"] is True
    for k in a["model"]:
        torch.testing.assert_close(a["model"][k].float(), s["model"][k].float(), rtol=2e-2, atol=2e-3)


# ---------------------------------------------------------------------------------------------
def _replica_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.parallel.consistency import replica_report

    torch.manual_seed(0)
    m = Transformer(get_preset("llama-micro", seq_len=64))
    flat = m.flatten_()
    opt = FlatAdamW(flat, lr=1e-3)
    ok = replica_report(flat, opt)
    if rank == 1:
        with torch.no_grad():
            flat.data[12345] += 1e-3  # one element of one replica
    bad = replica_report(flat, opt)
    if rank == 1:
        with torch.no_grad():
            flat.data[12345] -= 1e-3
            opt.exp_avg[7] = 1.0
    bad_opt = replica_report(flat, opt)
    torch.save({"ok": ok, "bad": bad, "bad_opt": bad_opt}, os.path.join(out_dir, f"rep_{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_replica_check_detects_a_perturbed_rank(tmp_path):
    """One rank changes one parameter element: every rank's report says the parameters differ;
    then one moment element: the optimizer state differs, the parameters agree again."""
    mp.spawn(_replica_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        rep = torch.load(os.path.join(tmp_path, f"rep_{r}.pt"), weights_only=False)
        assert rep["ok"]["params_identical_across_ranks"] and rep["ok"]["optimizer_identical_across_ranks"]
        assert rep["ok"]["mismatched"] == []
        assert not rep["bad"]["params_identical_across_ranks"] and rep["bad"]["mismatched"] == ["params"]
        assert rep["bad_opt"]["params_identical_across_ranks"]
        assert rep["bad_opt"]["optimizer_identical_across_ranks"] is False


def test_checksum_hash_definition():
    """The torch hash is sum_i w_i (2 i + 1) mod 2^64 over 32-bit words (the kernel's definition),
    and it changes when two words swap."""
    from pyrecover_amd.parallel.consistency import _hash_torch

    x = torch.tensor([1.5, -2.0, 3.25, 7.0], dtype=torch.float32)
    w = [int(v) & 0xFFFFFFFF for v in x.view(torch.int32).tolist()]
    assert _hash_torch(x) == sum(wi * (2 * i + 1) for i, wi in enumerate(w)) % 2**64
    assert _hash_torch(x) != _hash_torch(x[[1, 0, 2, 3]])


def test_bench_cpu_two_ranks_reports_identical_replicas():
    """bench.py W = 2 (gloo): the JSON line says the replicas are identical after the timed steps,
    with the sharded optimizer and the sparse embedding exchange on."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, PYRECOVER_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--cpu", "--model", "llama-micro", "--steps", "2",
           "--warmup", "1", "--batch-per-gpu", "2", "--seq-len", "64", "--bucket-mb", "0.05", "--shard-optimizer",
           "--sparse-embedding-grad", "on"]
    out = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    js = json.loads(line)
    assert js["params_identical_across_ranks"] is True and js["optimizer_identical_across_ranks"] is None
    assert js["config"]["shard_optimizer"] is True and js["config"]["sparse_embedding_grad"] is True


# ---------------------------------------------------------------------------------------------
def test_reduction_settings_record_bucket_and_mode(tmp_path):
    """A default W > 1 run records what it reduced with -- world size, backend, bucket MiB, ZeRO-1 /
    sparse flags, and that RCCL's order was NOT pinned (PYRECOVER_RCCL_DETERMINISTIC is opt-in) --
    and a resume under a different bucket size is reported as a difference."""
    from pyrecover_amd.ckpt import core as ckcore
    from pyrecover_amd.parallel import dist as D

    _run(2, _zargv(tmp_path, 2, ["--checkpoint-frequency", "2"]), tmp_path)
    path = tmp_path / "e" / "ckpt_2.pt"
    red = _state(path)["pyrecover_state"]["reduction"]
    assert red["world_size"] == 2 and red["backend"] == "gloo" and red["bucket_mb"] == 0.05
    assert red["rccl_order_pinned"] is False and red["shard_optimizer"] is False
    assert red["sparse_embedding"] is False and "NCCL_ALGO" not in red
    assert ckcore.peek_reduction(str(path)) == red
    assert ckcore.peek_reduction("latest", exp_dir=tmp_path / "e") == red
    cur = dict(red, bucket_mb=64.0)
    diffs = D.compare_rccl_order(red, cur)
    assert len(diffs) == 1 and diffs[0].startswith("bucket_mb")
    # a checkpoint of an older version (no bucket_mb / flags) is not a difference
    old = {k: v for k, v in red.items() if k not in D._NEWER_KEYS}
    assert D.compare_rccl_order(old, red) == []


def test_bucket_auto_resume_reuses_the_checkpointed_size(tmp_path):
    """--bucket-cap-mb auto on resume takes the bucket size the checkpoint was written with instead
    of probing again (the probe may choose differently on a new allocation)."""
    ex = ["--checkpoint-frequency", "2"]
    _run(2, _zargv(tmp_path, 2, ex + ["--bucket-cap-mb", "auto"]), tmp_path)
    first = _state(tmp_path / "e" / "ckpt_2.pt")["pyrecover_state"]["reduction"]["bucket_mb"]
    # rewrite the recorded size: the resumed run must use it (a probe would pick 16..512)
    ck = _state(tmp_path / "e" / "ckpt_2.pt")
    ck["pyrecover_state"]["reduction"]["bucket_mb"] = 0.25
    torch.save(ck, tmp_path / "e" / "ckpt_2.pt")
    _run(2, _zargv(tmp_path, 4, ex + ["--bucket-cap-mb", "auto", "--resume-from-checkpoint", "latest"]), tmp_path)
    assert 16 <= first <= 512
    assert _state(tmp_path / "e" / "ckpt_4.pt")["pyrecover_state"]["reduction"]["bucket_mb"] == 0.25


def test_checkpoint_bytes_counts_the_fp32_master(tmp_path):
    """the final-save estimate and the pinned pool are sized from the real state: with
    --master-weights fp32 the checkpoint holds bf16 params + fp32 m, v, master (14 B/param), and
    the bytes a save writes match FlatAdamW.checkpoint_bytes() (to the archive's small entries)."""
    from pyrecover_amd.ckpt.vanilla import save_ckpt_vanilla
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW

    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    m = Transformer(get_preset("llama-micro", seq_len=64))
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    for mw, per in ((False, 6), (True, 14)):
        opt = FlatAdamW(flat, lr=1e-3, master_weights=mw)
        nparam = sum(p.numel() for p in m.parameters())
        est = opt.checkpoint_bytes()
        assert abs(est - per * flat.numel) < 1e-9 * est + 1 and est >= per * nparam
        p = tmp_path / f"ckpt_{int(mw)}.pt"
        save_ckpt_vanilla(m, opt, None, None, 1, 1, str(p), max_keep=0, verify=False)
        size = p.stat().st_size
        assert per * nparam <= size <= per * nparam * 1.02 + (2 << 20), (mw, size, per * nparam)


def test_shard_optimizer_auto_policy():
    """--shard-optimizer auto: ZeRO-1 at W > 1 for a 16-bit GPU model that carries no transposed
    weight shadows at its batch (grouped-query attention at <= 4096 tokens per rank); never at
    W = 1, for CPU / fp32 models, or when the model keeps shadows; on / off / a bare flag override."""
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.trainer import _use_shard_optimizer

    gqa = Transformer(get_preset("llama-micro", seq_len=64))  # 2 heads, 1 kv head
    mha = Transformer(get_preset("llama-micro", seq_len=64, n_kv_heads=2))
    assert _use_shard_optimizer("auto", 8, gqa, 2048, True)
    assert not _use_shard_optimizer("auto", 8, gqa, 8192, True)  # shadows pay at 8192 tokens
    assert not _use_shard_optimizer("auto", 8, mha, 2048, True)
    assert not _use_shard_optimizer("auto", 1, gqa, 2048, True)
    assert not _use_shard_optimizer("auto", 8, gqa, 2048, False)  # CPU or fp32
    assert _use_shard_optimizer("on", 2, mha, 32768, False) and _use_shard_optimizer(True, 2, mha, 32768, True)
    assert not _use_shard_optimizer("off", 8, gqa, 2048, True)
