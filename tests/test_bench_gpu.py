"""bench.py's multi-rank launch on the GPU box: `python bench.py --gpus 2` (no torchrun, no rank
environment) must start 2 rank processes itself and report a 2-rank job. Both ranks share GPU 0
(PYRECOVER_LOCAL_DEVICE=0) and reduce over gloo, because RCCL refuses two ranks on one device; the
driver's N-GPU run takes the same code path with RCCL and one GPU per rank."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus2_spawns_two_ranks(cuda):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYRECOVER_LOCAL_DEVICE="0", PYRECOVER_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "gpt2-small",
                        "--batch-per-gpu", "2", "--steps", "3", "--warmup", "1", "--bucket-mb", "auto"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-5000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2, out
    assert out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]
    # N-GPU diagnostics recorded with HIP events
    c = out["comm"]
    assert c["timing_source"] == "hip events" and len(c["exposed_comm_ms_per_rank"]) == 2
    assert c["exposed_comm_ms"] >= 0 and c["allreduce_busy_ms"] > 0
    assert len(c["buckets"]) == out["config"]["grad_buckets"]
    assert all(b["ms"] >= 0 and b["mib"] > 0 for b in c["buckets"])
    assert "comm_env" in out
    # --bucket-mb auto: the startup probe ran on the 2-rank group and chose the bucket cap
    tune = out["config"]["bucket_autotune"]
    assert tune["world"] == 2 and tune["chosen_mb"] == out["config"]["bucket_mb"] and len(tune["probe"]) == 4


def test_bench_gpus2_sharded_optimizer_sparse_embedding_replicas_identical(cuda):
    """--shard-optimizer (reduce-scatter, 1/W AdamW update on the HIP kernel, parameter all-gather)
    with the sparse embedding exchange, 2 ranks on GPU 0 over gloo: the replicas are bitwise identical
    after the timed steps (the JSON says so; bench.py exits 3 otherwise), and the loss matches the
    all-reduce run's."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYRECOVER_LOCAL_DEVICE="0", PYRECOVER_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    outs = []
    for extra in ([], ["--shard-optimizer", "--sparse-embedding-grad", "on"]):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "gpt2-small",
                            "--batch-per-gpu", "2", "--steps", "3", "--warmup", "1", "--bucket-mb", "32",
                            "--sparse-embedding-grad", "off"] + extra,
                           capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
        assert r.returncode == 0, (r.stdout + r.stderr)[-5000:]
        line = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1]
        outs.append(json.loads(line))
    dense, zero = outs
    assert dense["params_identical_across_ranks"] and dense["optimizer_identical_across_ranks"]
    assert zero["params_identical_across_ranks"] and zero["optimizer_identical_across_ranks"] is None
    assert zero["config"]["shard_optimizer"] and zero["config"]["sparse_embedding_grad"]
    assert not zero["config"]["weight_shadows"]
    assert abs(zero["final_loss"] - dense["final_loss"]) < 0.05 * abs(dense["final_loss"]) + 1e-3


def test_bench_gpus2_auto_shards_a_gqa_batch1_job(cuda):
    """--shard-optimizer auto (the default): a grouped-query model at batch 1 carries no weight
    shadows, so a 2-rank job runs ZeRO-1 on its own, and its replicas end bitwise identical."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(PYRECOVER_LOCAL_DEVICE="0", PYRECOVER_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "llama-tiny",
                        "--batch-per-gpu", "1", "--seq-len", "256", "--steps", "3", "--warmup", "1",
                        "--bucket-mb", "0.25"], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-5000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')][-1])
    assert out["config"]["shard_optimizer"] is True and not out["config"]["weight_shadows"]
    assert out["params_identical_across_ranks"] is True


def test_replica_checksum_kernel_matches_torch(cuda):
    """pra_checksum (csrc/kernels/comm.hip) against the torch definition: the 64-bit word hash is
    exact, the fp64 element sum equal to rounding; one flipped bit changes the hash."""
    import torch

    from pyrecover_amd.parallel import consistency as C

    g = torch.Generator(device=cuda).manual_seed(7)
    for dt, n in ((torch.bfloat16, 1 << 20), (torch.float32, 3 * (1 << 18) + 64), (torch.bfloat16, 4096 * 8 + 8)):
        x = torch.randn(n, generator=g, device=cuda).to(dt)
        s, h = C.buffer_checksum(x)
        assert h == C._hash_torch(x.cpu())
        assert abs(s - C._sum_torch(x.cpu())) <= 1e-9 * x.double().abs().sum().item() + 1e-6
        y = x.clone()
        y.view(torch.int16)[12345] ^= 1
        assert C.buffer_checksum(y)[1] != h
