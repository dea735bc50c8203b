"""Multi-process (gloo, world_size 2) tests of the DDP engine and sharded checkpoints on CPU."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, argv, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    res = train(get_args(argv))
    torch.save(res, os.path.join(out_dir, f"res_{rank}.pt"))


def _run(world, argv, tmp):
    port = _free_port()
    if world == 1:
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            os.environ.pop(k, None)
        from pyrecover_amd.cli import get_args
        from pyrecover_amd.trainer import train

        return train(get_args(argv))
    mp.spawn(_worker, args=(world, port, argv, str(tmp)), nprocs=world, join=True)
    return torch.load(os.path.join(tmp, "res_0.pt"), weights_only=False)


def _argv(ckdir, steps, extra=()):
    return ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "4",
            "--training-steps", str(steps), "--checkpoint-dir", str(ckdir), "--experiment_name", "e",
            "--checkpoint-frequency", "2", "--model-dtype", "fp32", "--num-workers", "0", "--logging-frequency", "100",
            "--learning-rate", "1e-3", "--bucket-cap-mb", "0.05"] + list(extra)


def _model(path):
    return torch.load(path, weights_only=True)["model"]


def test_ddp_matches_single_process(tmp_path):
    """2 ranks x local batch 2 == 1 rank x batch 4 (same samples), up to fp32 reduction order."""
    _run(2, _argv(tmp_path / "ddp", 2, ["--distributed"]), tmp_path)
    _run(1, _argv(tmp_path / "single", 2), tmp_path)
    a = _model(tmp_path / "ddp" / "e" / "ckpt_2.pt")
    b = _model(tmp_path / "single" / "e" / "ckpt_2.pt")
    for k in a:
        assert torch.allclose(a[k], b[k], rtol=1e-4, atol=1e-5), (k, (a[k] - b[k]).abs().max())


def test_sharded_checkpoint_two_ranks_and_reshard(tmp_path):
    ck = tmp_path / "ck"
    _run(2, _argv(ck, 2, ["--distributed", "--use-torch-distributed-ckpt"]), tmp_path)
    d = ck / "e" / "ckpt_2"
    files = sorted(x.name for x in d.iterdir())
    assert "__0_0.distcp" in files and "__1_0.distcp" in files and ".metadata" in files
    sizes = [(d / f).stat().st_size for f in ("__0_0.distcp", "__1_0.distcp")]
    assert min(sizes) > 0.3 * max(sizes), sizes  # byte-balanced shards
    # world-size agnostic: resume the 2-rank sharded checkpoint in a single process
    r = _run(1, _argv(ck, 4, ["--use-torch-distributed-ckpt", "--resume-from-checkpoint", "latest"]), tmp_path)
    assert r["step"] == 4


def test_ddp_resume_bit_exact(tmp_path):
    """2-rank run preempted at step 3 and resumed == uninterrupted 2-rank run (tolerance 0)."""
    _run(2, _argv(tmp_path / "a", 4, ["--distributed"]), tmp_path)
    _run(2, _argv(tmp_path / "b", 4, ["--distributed", "--stop-at-step", "3"]), tmp_path)
    _run(2, _argv(tmp_path / "b", 4, ["--distributed", "--resume-from-checkpoint", "latest"]), tmp_path)
    a = torch.load(tmp_path / "a" / "e" / "ckpt_4.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "e" / "ckpt_4.pt", weights_only=True)
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        assert torch.equal(a["optimizer"]["state"][i]["exp_avg_sq"], b["optimizer"]["state"][i]["exp_avg_sq"])


def _worker_slurm(rank, world, port, argv, out_dir, end_in_s):
    """A rank started by srun: only SLURM_* variables (no torchrun env)."""
    import time

    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        os.environ.pop(k, None)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), SLURM_PROCID=str(rank),
                      SLURM_NTASKS=str(world), SLURM_LOCALID=str(rank), SLURM_JOB_ID="4242")
    if end_in_s is not None:
        os.environ["SLURM_JOB_END_TIME"] = str(time.time() + end_in_s)
    else:
        os.environ.pop("SLURM_JOB_END_TIME", None)
    torch.set_num_threads(2)
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    res = train(get_args(argv))
    torch.save(res, os.path.join(out_dir, f"res_{rank}.pt"))


def test_fake_slurm_two_ranks_timeaware_stop_and_resume(tmp_path):
    """2 gloo ranks bootstrapped from fake SLURM variables (SLURM_PROCID/NTASKS/LOCALID) and
    a SLURM_JOB_END_TIME 30 s away: rank 0 decides to stop at step 1, its flag (broadcast without a
    per-step host sync, read one step later: SURVEY D16) stops both ranks after step 2, they write
    the final sharded checkpoint, and a second fake-SLURM job resumes it to completion."""
    ck = tmp_path / "ck"
    argv = _argv(ck, 6, ["--distributed", "--use-torch-distributed-ckpt", "--timeaware-checkpointing",
                         "--checkpoint-frequency", "-1"])
    mp.spawn(_worker_slurm, args=(2, _free_port(), argv, str(tmp_path), 30.0), nprocs=2, join=True)
    r0 = torch.load(tmp_path / "res_0.pt", weights_only=False)
    r1 = torch.load(tmp_path / "res_1.pt", weights_only=False)
    assert r0["stopped_early"] and r1["stopped_early"] and r0["step"] == r1["step"] == 2
    assert (ck / "e" / "ckpt_2_final" / ".metadata").exists()
    argv2 = _argv(ck, 3, ["--distributed", "--use-torch-distributed-ckpt", "--resume-from-checkpoint", "latest"])
    mp.spawn(_worker_slurm, args=(2, _free_port(), argv2, str(tmp_path), None), nprocs=2, join=True)
    assert torch.load(tmp_path / "res_0.pt", weights_only=False)["step"] == 3


@pytest.mark.parametrize("batch", [1, 3])
def test_tokens_per_second_counts_what_runs(tmp_path, batch):
    """with --batch-size not a multiple of W the reference logs B·S tokens per step
    (train.py:252) while each rank runs max(B//W,1) sequences (:62-63). Here the logged tokens/s
    must match the tokens that actually ran (local 1 x W 2 x S) over the measured step time."""
    import json

    ck = tmp_path / "ck"
    seq = 128
    jl = tmp_path / "m.jsonl"
    argv = _argv(ck, 8, ["--distributed", "--checkpoint-frequency", "-1", "--logging-frequency", "1",
                         "--metrics-jsonl", str(jl)])
    argv[argv.index("--batch-size") + 1] = str(batch)
    _run(2, argv, tmp_path)
    recs = [json.loads(ln) for ln in open(jl)]
    assert [r["step"] for r in recs] == list(range(1, 9))
    per_step = 1 * 2 * seq  # local batch max(B//2,1) = 1 on each of 2 ranks
    ratios = sorted(r["tokens_per_s"] * (r["time"] - p["time"]) / per_step for p, r in zip(recs[1:], recs[2:]))
    med = ratios[len(ratios) // 2]
    assert 0.9 < med < 1.1, ratios
    assert all(abs(r["tokens_per_s_per_gpu"] * 2 - r["tokens_per_s"]) < 1e-6 * r["tokens_per_s"] for r in recs)


def _bench_json(out: str) -> dict:
    import json

    lines = [ln for ln in out.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_self_spawns_ranks():
    """`python bench.py --gpus 2` without a rank environment starts 2 ranks itself (no silent 1-GPU
    number); the JSON line reports n_gpus == ranks_seen == 2."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu", "--model",
                        "llama-micro", "--seq-len", "64", "--batch-per-gpu", "2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2, out
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 4
    assert out["config"]["dist_backend"] == "gloo"
    # N-GPU diagnostics (exposed communication, per-bucket all-reduce time/bandwidth, RCCL env)
    c = out["comm"]
    assert c["exposed_comm_ms"] >= 0 and len(c["exposed_comm_ms_per_rank"]) == 2
    assert len(c["buckets"]) == out["config"]["grad_buckets"] and c["allreduce_busy_ms"] > 0
    assert all(b["ms"] >= 0 and b["mib"] > 0 for b in c["buckets"])
    assert isinstance(out["comm_env"], dict)


def test_bench_rejects_world_mismatch():
    """A rank environment whose world size differs from --gpus is an error, not a 1-GPU number."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu", "--model",
                        "llama-micro", "--seq-len", "64", "--batch-per-gpu", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert '"metric"' not in r.stdout


def test_bench_launch_command():
    import bench

    cmd = bench.launch_command(["--gpus", "8", "--steps", "3"], 8, {})
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-3:] == ["--gpus", "8", "--steps", "3"][-3:]
    assert bench.launch_command(["--gpus", "8"], 8, {"WORLD_SIZE": "8"}) == []
    assert bench.launch_command([], 1, {}) == []
    assert bench.launch_command(["--gpus", "4"], 4, {"SLURM_PROCID": "0", "SLURM_NTASKS": "4"}) == []


def _hostseq_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from pyrecover_amd.parallel.xgmi import _HostSeq

    dist.init_process_group("gloo", rank=rank, world_size=world)
    hs = _HostSeq(rank, world, 3, None)
    name = hs.shm.name
    for seq in range(1, 51):  # ping-pong: each slot published then awaited by every peer
        for slot in range(3):
            hs.publish(slot, seq)
            for r in range(world):
                hs.wait(r, slot, seq, timeout=30)
    dist.barrier()
    hs.close()
    dist.barrier()
    with open(os.path.join(out_dir, f"hs_{rank}.txt"), "w") as f:
        f.write(f"{name} {os.path.exists('/dev/shm/' + name)}")
    dist.destroy_process_group()


def test_xgmi_host_sequence_words(tmp_path):
    """The shared-memory sequence words that order the xGMI backend's IPC events (no gloo barrier
    per bucket): 2 processes, 150 publish/wait rounds, segment unlinked after close."""
    mp.spawn(_hostseq_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        name, exists = open(tmp_path / f"hs_{r}.txt").read().split()
        assert name.startswith("pra_xgmi_") and exists == "False"


def test_bench_cpu_overlapped_optimizer_many_buckets():
    """Overlapped AdamW updates bucket by bucket DURING backward; on the CPU path this must not
    bump the flat buffer's autograd version counter (it invalidated saved weights of layers whose
    backward had not run yet)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--cpu", "--model",
                        "llama-micro", "--seq-len", "64", "--batch-per-gpu", "2", "--steps", "2", "--warmup", "1",
                        "--bucket-mb", "0.02"], capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _bench_json(r.stdout)
    assert out["config"]["grad_buckets"] > 3 and len(out["comm"]["buckets"]) == out["config"]["grad_buckets"]


def _rng_worker(rank, world, port, out_dir, fmt):
    import random

    import torch.distributed as dist

    from pyrecover_amd.ckpt import sharded, vanilla

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.set_num_threads(1)
    torch.manual_seed(0)
    model = torch.nn.Linear(8, 8)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    model(torch.randn(2, 8)).sum().backward()
    opt.step()
    torch.manual_seed(100 + rank)  # every rank its own streams
    random.seed(7 * rank + 1)
    path = os.path.join(out_dir, "ckpt_1.pt" if fmt == "vanilla" else "ckpt_1")
    save = vanilla.save_ckpt_vanilla if fmt == "vanilla" else sharded.save_ckpt_distributed
    load = vanilla.load_ckpt_vanilla if fmt == "vanilla" else sharded.load_ckpt_distributed
    save(model, opt, step=1, epoch=1, checkpoint_path=path, verify=False, is_distributed=True, rank=rank)
    want = (torch.rand(4), random.random())
    torch.manual_seed(999)
    random.seed(999)
    load(model, opt, checkpoint_path=path, experiment_dir=out_dir, verify=False, is_distributed=True, rank=rank)
    got = (torch.rand(4), random.random())
    torch.save({"want": want, "got": got}, os.path.join(out_dir, f"rng_{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("fmt", ["vanilla", "sharded"])
def test_checkpoint_restores_each_ranks_own_rng(tmp_path, fmt):
    """Every rank's RNG streams are saved (pyrecover_state.rng_per_rank) and each rank restores its
    own, not the saving rank's (reference saves none)."""
    mp.spawn(_rng_worker, args=(2, _free_port(), str(tmp_path), fmt), nprocs=2, join=True)
    r = [torch.load(tmp_path / f"rng_{i}.pt", weights_only=False) for i in range(2)]
    for x in r:
        assert torch.equal(x["want"][0], x["got"][0]) and x["want"][1] == x["got"][1]
    assert not torch.equal(r[0]["got"][0], r[1]["got"][0])
    if fmt == "vanilla":  # the reference key set is untouched; the extra entry rides along
        ck = torch.load(tmp_path / "ckpt_1.pt", weights_only=False)
        assert {"epoch", "step", "model", "optimizer"} <= set(ck)
        assert len(ck["pyrecover_state"]["rng_per_rank"]) == 2


def test_xgmi_visibility_check_compares_device_identity():
    """Per-task isolation (each rank sees only its own GPU as index 0) is refused; ranks sharing one
    GPU (one-GPU rehearsal) and a node with every GPU visible pass."""
    from pyrecover_amd.parallel.xgmi import _hidden_ranks

    assert _hidden_ranks([("A", ["A"]), ("B", ["B"])]) == [0, 1]
    assert _hidden_ranks([("A", ["A"]), ("A", ["A"])]) == []
    assert _hidden_ranks([("A", ["A", "B"]), ("B", ["A", "B"])]) == []
    assert _hidden_ranks([("A", ["A", "B"]), ("B", ["B"])]) == [0]


def test_metrics_jsonl_diagnostics_two_ranks(tmp_path):
    """SURVEY §5.5 / reference train.py:283-296: every JSONL log record of a 2-rank gloo run carries
    the device step time, HBM usage, the exposed all-reduce time with its bus bandwidth, and the
    checkpoint stall / background write time (null where the quantity does not exist on CPU)."""
    import json

    ck = tmp_path / "ck"
    jl = tmp_path / "m.jsonl"
    argv = _argv(ck, 6, ["--distributed", "--checkpoint-frequency", "2", "--logging-frequency", "2",
                         "--metrics-jsonl", str(jl), "--timeaware-checkpointing"])
    _run(2, argv, tmp_path)
    recs = [json.loads(ln) for ln in open(jl)]
    assert [r["step"] for r in recs] == [1, 2, 4, 6]
    keys = {"device_step_ms", "device_step_max_ms", "hbm_gib", "hbm_peak_gib", "hbm_reserved_gib",
            "exposed_comm_ms", "allreduce_busy_ms", "allreduce_busbw_gbps", "ckpt_saves", "ckpt_stall_s",
            "ckpt_write_s", "ckpt_write_gib", "max_iter_time_s", "ckpt_budget_s", "stop_threshold_s"}
    for r in recs:
        assert keys <= set(r), keys - set(r)
        assert r["exposed_comm_ms"] is not None and r["exposed_comm_ms"] >= 0
        assert r["allreduce_busy_ms"] > 0 and r["allreduce_busbw_gbps"] > 0
    assert recs[2]["ckpt_saves"] == 1 and recs[2]["ckpt_stall_s"] > 0  # the save at step 4 ...
    assert any(r["ckpt_write_s"] for r in recs[2:])  # ... and a completed background write


# ---------------------------------------------------------------------------------------------
# World size 4 (gloo): more than two owners / reducers, resharding 4 -> 2, the stop flag at W=4


def test_ddp_w4_resume_bit_exact_and_matches_single(tmp_path):
    """4 ranks (local batch 1 each): a run preempted at step 3 and resumed is bit-identical to an
    uninterrupted one (tolerance 0): weights and both AdamW moments. (Against one process on the same
    global batch the result differs by design, as with the reference's DDP: each rank averages its
    own tokens' loss before the gradient all-reduce averages the ranks.)"""
    _run(4, _argv(tmp_path / "a", 4, ["--distributed"]), tmp_path)
    _run(4, _argv(tmp_path / "b", 4, ["--distributed", "--stop-at-step", "3"]), tmp_path)
    _run(4, _argv(tmp_path / "b", 4, ["--distributed", "--resume-from-checkpoint", "latest"]), tmp_path)
    a = torch.load(tmp_path / "a" / "e" / "ckpt_4.pt", weights_only=True)
    b = torch.load(tmp_path / "b" / "e" / "ckpt_4.pt", weights_only=True)
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    for i in a["optimizer"]["state"]:
        for key in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(a["optimizer"]["state"][i][key], b["optimizer"]["state"][i][key]), (i, key)


def test_sharded_w4_owners_reshard_to_w2(tmp_path):
    """A sharded checkpoint written by 4 owners has 4 byte-balanced shard files and the same content
    as the vanilla checkpoint of the same run; it resumes at world size 2 (4 -> 2 resharding)."""
    import sys

    ck = tmp_path / "sh"
    _run(4, _argv(ck, 2, ["--distributed", "--use-torch-distributed-ckpt"]), tmp_path)
    d = ck / "e" / "ckpt_2"
    shards = sorted(d.glob("__*_0.distcp"))
    assert [p.name for p in shards] == [f"__{r}_0.distcp" for r in range(4)]
    sizes = [p.stat().st_size for p in shards]
    assert min(sizes) > 0.5 * max(sizes), sizes
    _run(4, _argv(tmp_path / "va", 2, ["--distributed"]), tmp_path)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "tools"))
    from check_weights_equality import main as weq

    assert weq([str(tmp_path / "va" / "e" / "ckpt_2.pt"), str(d), "--distributed", "--optimizer"]) == 0
    r = _run(2, _argv(ck, 3, ["--distributed", "--use-torch-distributed-ckpt", "--resume-from-checkpoint",
                              "latest"]), tmp_path)
    assert r["step"] == 3


def test_w4_timeaware_stop_flag_uneven_batch(tmp_path):
    """4 fake-SLURM ranks, --batch-size 6 (not a multiple of W: each rank runs 1 sequence), a limit
    30 s away: rank 0 decides at step 1, every rank acts on the broadcast one step later (step 2),
    the final sharded checkpoint has 4 shards, and the job resumes from it."""
    ck = tmp_path / "ck"
    argv = _argv(ck, 6, ["--distributed", "--use-torch-distributed-ckpt", "--timeaware-checkpointing",
                         "--checkpoint-frequency", "-1"])
    argv[argv.index("--batch-size") + 1] = "6"
    mp.spawn(_worker_slurm, args=(4, _free_port(), argv, str(tmp_path), 30.0), nprocs=4, join=True)
    res = [torch.load(tmp_path / f"res_{r}.pt", weights_only=False) for r in range(4)]
    assert all(x["stopped_early"] and x["step"] == 2 for x in res), res
    fin = ck / "e" / "ckpt_2_final"
    assert (fin / ".metadata").exists() and len(list(fin.glob("__*_0.distcp"))) == 4
    argv2 = _argv(ck, 3, ["--distributed", "--use-torch-distributed-ckpt", "--resume-from-checkpoint", "latest"])
    argv2[argv2.index("--batch-size") + 1] = "6"
    mp.spawn(_worker_slurm, args=(4, _free_port(), argv2, str(tmp_path), None), nprocs=4, join=True)
    assert torch.load(tmp_path / "res_0.pt", weights_only=False)["step"] == 3


# ---------------------------------------------------------------------------------------------
# Bucket-size autotune (parallel/bucket_tune.py)


def test_bucket_tune_fit_and_choice():
    from pyrecover_amd.parallel.bucket_tune import choose_bucket_mb, fit_latency_bandwidth, parse_bucket_arg

    mib = 2 ** 20
    # t = 30 us + s / 150 GB/s, exactly
    samples = [(s * mib, 30e-6 + s * mib / 150e9) for s in (4, 16, 64, 256)]
    a, b = fit_latency_bandwidth(samples)
    assert a == pytest.approx(30e-6, rel=1e-6) and b == pytest.approx(150e9, rel=1e-6)
    # alpha <= 10% of t(s)  <=>  s >= 9 alpha beta = 40.5 MB = 38.6 MiB -> 64 MiB (powers of two from 16)
    assert choose_bucket_mb(a, b) == 64
    assert choose_bucket_mb(1e-3, 150e9) == 512  # clamped at hi
    assert choose_bucket_mb(0.0, 150e9) == 16 and choose_bucket_mb(1e-5, float("inf")) == 16
    assert parse_bucket_arg("auto") == "auto" and parse_bucket_arg("32") == 32.0
    with pytest.raises(ValueError):
        parse_bucket_arg("-1")


def _tune_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from pyrecover_amd.parallel.bucket_tune import autotune_bucket_mb

    mb, rep = autotune_bucket_mb(torch.device("cpu"), torch.float32, sizes_mb=(1, 2, 4), iters=2)
    torch.save({"mb": mb, "rep": rep}, os.path.join(out_dir, f"tune_{rank}.pt"))
    torch.distributed.destroy_process_group()


def test_bucket_autotune_two_ranks_agree(tmp_path):
    """The probe runs on the job's group, every rank ends with rank 0's choice, and the report carries
    the fitted latency / bandwidth and the per-size times."""
    mp.spawn(_tune_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (torch.load(os.path.join(tmp_path, f"tune_{r}.pt"), weights_only=False) for r in (0, 1))
    assert r0["mb"] == r1["mb"] and 16 <= r0["mb"] <= 512
    rep = r0["rep"]
    assert rep["world"] == 2 and rep["chosen_mb"] == r0["mb"] and len(rep["probe"]) == 3
    assert all(p["ms"] > 0 for p in rep["probe"])


def test_train_bucket_cap_auto_two_ranks(tmp_path):
    """--bucket-cap-mb auto end to end (train.py, 2 gloo ranks)."""
    argv = _argv(tmp_path / "ck", 2, ["--distributed"])
    argv[argv.index("--bucket-cap-mb") + 1] = "auto"
    res = _run(2, argv, tmp_path)
    assert res is not None


def test_fp32_master_two_ranks_sharded_resume_and_reshard(tmp_path):
    """--master-weights fp32 at W=2 with sharded checkpoints: the owners write the master next to the
    moments, a preempted-and-resumed 2-rank run is bit-identical to an uninterrupted one (master
    included), and the 2-rank checkpoint resumes in a single process (2 -> 1 resharding)."""
    from pyrecover_amd.ckpt.sharded import read_sharded_state

    extra = ["--distributed", "--use-torch-distributed-ckpt", "--model-dtype", "bf16", "--master-weights", "fp32"]
    _run(2, _argv(tmp_path / "a", 4, extra), tmp_path)
    _run(2, _argv(tmp_path / "b", 4, extra + ["--stop-at-step", "3"]), tmp_path)
    _run(2, _argv(tmp_path / "b", 4, extra + ["--resume-from-checkpoint", "latest"]), tmp_path)
    a = read_sharded_state(str(tmp_path / "a" / "e" / "ckpt_4"))
    b = read_sharded_state(str(tmp_path / "b" / "e" / "ckpt_4"))
    for k in a["model"]:
        assert torch.equal(a["model"][k], b["model"][k]), k
    sa, sb = a["optimizer"]["state"], b["optimizer"]["state"]
    assert sa and all("master_param" in v for v in sa.values())
    for i in sa:
        for key in ("master_param", "exp_avg", "exp_avg_sq"):
            assert sa[i][key].dtype == torch.float32 and torch.equal(sa[i][key], sb[i][key]), (i, key)
    r = _run(1, _argv(tmp_path / "a", 6, ["--use-torch-distributed-ckpt", "--model-dtype", "bf16", "--master-weights",
                                          "fp32", "--resume-from-checkpoint", "latest"]), tmp_path)
    assert r["step"] == 6
