"""CPU tests of the framework around the kernels: CLI parity, data, sampler, LR schedule,
time-aware stop (fake clock), resubmission, retention/latest, tools, fault injection."""
import os
import subprocess
import sys
import time
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]

REFERENCE_FLAGS = {  # flag -> reference default (reference utils.py:105-261)
    "dataset": "/capstor/store/cscs/ethz/large-sc/datasets/train_data.parquet",
    "tokenizer_name_or_path": "unsloth/Mistral-Nemo-Base-2407-bnb-4bit",
    "sequence_length": 2048, "batch_size": 1, "fused_optimizer": False, "learning_rate": 1e-5,
    "lr_warmup_steps": 10, "training_steps": 1000, "logging_frequency": 5, "profile": False,
    "profile_step_start": 10, "profile_step_end": 12, "grad_max_norm": 1, "model_dtype": "bf16",
    "compile": False, "distributed": False, "checkpoint_dir": "checkpoints/", "checkpoint_frequency": 10,
    "resume_from_checkpoint": None, "experiment_name": "default-exp", "verify_checkpoints": False,
    "max_kept_checkpoints": 3, "use_torch_distributed_ckpt": False, "default_iter_time": 1.0,
    "default_ckpt_time": 10.0, "timeaware_checkpointing": False, "use_flash_attention": False,
    "log_loss_to_csv": False,
}


def test_cli_has_every_reference_flag_with_same_default():
    from pyrecover_amd.cli import get_args

    a = get_args([])
    for k, v in REFERENCE_FLAGS.items():
        assert getattr(a, k) == v, k
    a = get_args(["--experiment_name", "x", "--use_flash_attention", "--resume-from-checkpoint", "latest",
                  "--use-torch-distributed-ckpt", "--timeaware-checkpointing", "--model-dtype", "fp16"])
    assert a.experiment_name == "x" and a.use_flash_attention and a.resume_from_checkpoint == "latest"
    assert len(REFERENCE_FLAGS) == 28


def test_param_count_matches_reference_default():
    sys.path.insert(0, str(ROOT))
    import test_model

    assert test_model.main() == 8_053_329_920  # SURVEY §6 (derived from the reference model)


def test_lr_schedule_matches_reference():
    from pyrecover_amd.optim.lr import linear_warmup_constant

    assert [linear_warmup_constant(10, s) for s in (0, 4, 9, 10, 100)] == [1 / 11, 5 / 11, 10 / 11, 1, 1]


def test_collator_and_parquet_dataset(tmp_path):
    from pyrecover_amd.data.dataset import CollatorForCLM, ParquetDataset, make_synthetic_parquet
    from pyrecover_amd.data.tokenizer import ByteTokenizer

    p = make_synthetic_parquet(str(tmp_path / "d.parquet"), n_docs=5, min_words=1, max_words=40)
    tok = ByteTokenizer()
    ds = ParquetDataset(p, tok, 64, 12)
    assert len(ds) == 12
    assert ds[7]["input_ids"] == ds[2]["input_ids"]  # idx % real_length
    x, y = CollatorForCLM(64, tok.pad_token_id)([ds[i] for i in range(3)])
    assert x.shape == y.shape == (3, 64)
    assert ((y == -100) | (y != tok.pad_token_id)).all()
    full = torch.tensor([ds[0]["input_ids"]])
    assert torch.equal(x[0], full[0, :-1])


def test_sampler_is_deterministic_sharded_and_resumable():
    from pyrecover_amd.data.sampler import ResumableDistributedSampler

    s0 = ResumableDistributedSampler(10, 2, 0, seed=3)
    s1 = ResumableDistributedSampler(10, 2, 1, seed=3)
    a, b = list(s0), list(s1)
    assert sorted(a + b) == list(range(10))
    s0.advance(3)
    st = s0.state_dict()
    s2 = ResumableDistributedSampler(10, 2, 0, seed=3)
    s2.load_state_dict(st)
    assert list(s2) == a[3:]
    s2.set_epoch(1)
    assert list(s2) != a and s2.cursor == 0
    assert hasattr(s0, "set_state")  # stored under the reference's "sampler_state" key


def test_timeaware_stopper_reference_thresholds():
    from pyrecover_amd.timelimit import TimeAwareStopper

    now = [1000.0]
    st = TimeAwareStopper(1.0, 10.0, end_time=1100.0, clock=lambda: now[0])
    assert st.threshold == 1 + 10 + (10 * 1 + 2 * 10)  # 41 s initially
    assert not st.should_stop()
    st.update_iter(3.0)
    assert st.buffer == 5 * 3 + 10 and st.threshold == 3 + 10 + 25
    now[0] = 1100 - 37.9
    assert st.should_stop()
    st2 = TimeAwareStopper(1.0, 10.0, end_time=None)
    assert not st2.should_stop()
    st2.signaled = True
    assert st2.should_stop()


def test_timeaware_training_stops_and_resumes(tmp_path, monkeypatch):
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    # a job that "ends" in 30 s: below the 41 s initial threshold at step 1
    monkeypatch.setenv("SLURM_JOB_END_TIME", str(time.time() + 30))
    base = ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "2",
            "--training-steps", "50", "--checkpoint-dir", str(tmp_path), "--checkpoint-frequency", "-1",
            "--model-dtype", "fp32", "--num-workers", "0", "--timeaware-checkpointing", "--verify-checkpoints"]
    r = train(get_args(base))
    assert r["stopped_early"] and r["step"] == 1
    final = tmp_path / "default-exp" / "ckpt_1_final.pt"
    assert final.exists() and Path(str(final) + ".md5").exists()
    monkeypatch.delenv("SLURM_JOB_END_TIME")
    r = train(get_args(base[:-2] + ["--training-steps", "3", "--resume-from-checkpoint", "latest"]))
    assert r["step"] == 3 and not r["stopped_early"]


def test_timeaware_final_checkpoint_carries_md5_and_budgets_digest(tmp_path, monkeypatch):
    """The time-aware final checkpoint is written with its whole-file .md5 (inline, not a deferred
    digest that the wall-clock limit may cut short), the stop threshold budgets the final save's
    predicted cost, and an older checkpoint whose deferred digest was cut short is not left on
    disk without its .md5. Checked with the reference's own verification logic
    (pyrecover/checkpoint.py:157-171: md5 of the whole file == the sidecar's text)."""
    import hashlib

    from pyrecover_amd.ckpt import core as ckcore
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    end = time.time() + 300  # far above the initial 41 s threshold ...
    monkeypatch.setenv("SLURM_JOB_END_TIME", str(end))
    # ... until the first save completes and the measured rates predict a 400 s final save
    monkeypatch.setattr(ckcore.SaveCostModel, "final_seconds",
                        lambda self, nbytes=None: 400.0 if ckcore.WRITE_STATS["max_seconds"] > 0 else 0.0)
    monkeypatch.setitem(ckcore.WRITE_STATS, "max_seconds", 0.0)
    monkeypatch.setattr(ckcore, "_FLUSH_AT_EXIT", [True])  # abandon_deferred_md5 clears it

    def limit_reached(deadline=None):  # every deferred digest still running is abandoned
        ckcore.abandon_deferred_md5()
        return False

    monkeypatch.setattr(ckcore, "flush_all", limit_reached)
    args = ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "2",
            "--training-steps", "50", "--checkpoint-dir", str(tmp_path), "--checkpoint-frequency", "2",
            "--model-dtype", "fp32", "--num-workers", "0", "--timeaware-checkpointing", "--verify-checkpoints"]
    r = train(get_args(args))
    assert r["stopped_early"] and r["step"] == 3, r
    final = tmp_path / "default-exp" / "ckpt_3_final.pt"
    side = Path(str(final) + ".md5")
    assert side.exists() and side.stat().st_mtime < end
    with open(final, "rb") as f:
        assert hashlib.md5(f.read()).hexdigest() == side.read_text()
    for ck in (tmp_path / "default-exp").glob("ckpt_*.pt"):  # nothing unverifiable is kept
        assert Path(str(ck) + ".md5").exists(), ck


def test_timeaware_budget_sound_without_any_completed_save():
    """No save has completed before the stop (BASELINE config 4 with --checkpoint-frequency 1000
    and a 15-min limit). The reference budgets the final save at the 10 s prior; a 7B state
    (37.65 GiB) written with its inline serial MD5 takes ~40 s. The byte-based estimate makes the
    stop fire early enough; the prior alone would overrun the limit. Fake clock, 1.05 s steps."""
    from pyrecover_amd.ckpt.core import SaveCostModel
    from pyrecover_amd.timelimit import TimeAwareStopper

    state = int(37.65 * 2**30)
    cost = SaveCostModel(state, inline_md5=True, d2h_gbps=20.0)
    cost.probe_write_bps, cost.probe_md5_bps = 4.2e9, 0.96e9  # what the probes measure on the box
    est = cost.final_seconds()
    actual_final = state / 1.0e9 + 1.0  # mocked: MD5 a little slower than probed, plus overhead
    assert actual_final < est

    def run(with_estimate: bool):
        now = [0.0]
        end = 600.0
        st = TimeAwareStopper(1.0, 10.0, end_time=end, clock=lambda: now[0])
        if with_estimate:
            st.set_ckpt_estimate(est)
        step = 0
        while True:
            step += 1
            if st.should_stop():
                break
            now[0] += 1.05  # one step
            st.update_iter(1.05)
        return now[0] + 1.05 + actual_final, end  # the stop step, then the final save

    finish, end = run(True)
    assert finish < end, (finish, end)
    finish_prior, _ = run(False)
    assert finish_prior > end  # the reference's prior alone overruns


def test_step_timer_ignores_host_drain_on_log_steps(monkeypatch):
    """The iteration time is the device step, not the host span: a log step whose .item() drains
    6 queued steps (6 s of host wait) still reports ~1 s, and the interval spanning a checkpoint
    save's host pause is dropped."""
    from pyrecover_amd import trainer

    clock = {"dev": 0.0}
    done_at = []

    class FakeEvent:
        def __init__(self, enable_timing=False):
            self.t = None

        def record(self):
            clock["dev"] += 1.0  # every step takes 1.0 s of device time after the previous one
            self.t = clock["dev"]
            done_at.append(self)

        def query(self):
            return self.t <= clock["host"]

        def elapsed_time(self, other):
            return (other.t - self.t) * 1000.0

    monkeypatch.setattr(trainer.torch.cuda, "Event", FakeEvent)
    tm = trainer._StepTimer(True)
    clock["host"] = 0.0
    seen = []
    for step in range(1, 13):
        clock["host"] += 0.05  # host runs ahead
        if step % 6 == 0:
            clock["host"] = clock["dev"] + 1.0  # log step: .item() drains the queue
        seen.append(tm.record())
    assert max(seen) == pytest.approx(1.0)
    tm.gap()  # a save pauses the host for 30 s: the device idles
    clock["dev"] += 30.0
    clock["host"] = clock["dev"] + 5
    assert tm.record() == 0.0  # the interval spanning the pause is dropped
    clock["host"] += 2.0
    assert tm.record() == pytest.approx(1.0)
    mean, mx, n = tm.window()
    assert n >= 10 and mx == pytest.approx(1.0) and mean == pytest.approx(1.0)


def test_slurm_duration_parse_and_remaining(monkeypatch):
    from pyrecover_amd.timelimit import _parse_slurm_duration, get_remaining_time

    assert _parse_slurm_duration("1-02:03:04") == 86400 + 7384
    assert _parse_slurm_duration("39:30") == 2370
    assert _parse_slurm_duration("UNLIMITED") is None
    monkeypatch.setenv("SLURM_JOB_END_TIME", "2000")
    assert get_remaining_time(now=1500) == 500


def test_resubmit_commands():
    from pyrecover_amd.resubmit import ResubmitConfig, resubmit_command

    env = {"SLURM_JOB_ID": "77"}
    assert resubmit_command(ResubmitConfig("requeue"), env) == ["scontrol", "requeue", "77"]
    cmd = resubmit_command(ResubmitConfig("chain", "run.sh", ["--continue"]), env)
    assert cmd[:2] == ["sbatch", "--dependency=afterany:77"] and cmd[-2:] == ["run.sh", "--continue"]
    assert resubmit_command(ResubmitConfig("requeue"), {}) is None
    # requeue counts SLURM's own restart counter (scontrol requeue never changes our variable)
    assert resubmit_command(ResubmitConfig("requeue", max_resubmits=2),
                            {"SLURM_JOB_ID": "1", "SLURM_RESTART_COUNT": "2"}) is None
    assert resubmit_command(ResubmitConfig("requeue", max_resubmits=2),
                            {"SLURM_JOB_ID": "1", "SLURM_RESTART_COUNT": "1"}) == ["scontrol", "requeue", "1"]
    assert resubmit_command(ResubmitConfig("chain", "r.sh", max_resubmits=2),
                            {"SLURM_JOB_ID": "1", "PYRECOVER_RESUBMIT_COUNT": "2"}) is None


def test_retention_is_numeric_and_latest_skips_incomplete(tmp_path):
    from pyrecover_amd.ckpt.core import apply_retention, get_latest_checkpoint

    for s in (2000, 10000, 300):
        (tmp_path / f"ckpt_{s}.pt").write_bytes(b"x")
        (tmp_path / f"ckpt_{s}.pt.md5").write_text("0" * 32)
    apply_retention(tmp_path, 2, distributed=False)
    assert sorted(p.name for p in tmp_path.glob("*.pt")) == ["ckpt_10000.pt", "ckpt_2000.pt"]
    assert not (tmp_path / "ckpt_300.pt.md5").exists()
    d1, d2 = tmp_path / "ckpt_5", tmp_path / "ckpt_6"
    d1.mkdir()
    (d1 / ".metadata").write_bytes(b"m")
    d2.mkdir()
    (d2 / ".metadata").write_bytes(b"m")
    (d2 / ".incomplete").write_text("")
    assert get_latest_checkpoint(str(tmp_path), distributed=True) == str(d1)


def _tiny_run(ckdir, steps, extra=()):
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    return train(get_args(["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128",
                           "--batch-size", "2", "--training-steps", str(steps), "--checkpoint-dir", str(ckdir),
                           "--checkpoint-frequency", "2", "--model-dtype", "fp32", "--num-workers", "0"]
                          + list(extra)))


def test_weights_equality_tool(tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    from check_weights_equality import main

    _tiny_run(tmp_path / "a", 2)
    _tiny_run(tmp_path / "b", 2)
    _tiny_run(tmp_path / "c", 4)
    a, b, c = (str(tmp_path / x / "default-exp" / "ckpt_2.pt") for x in "abc")
    assert main([a, b, "--optimizer"]) == 0
    assert main([a, str(tmp_path / "c" / "default-exp" / "ckpt_4.pt")]) == 1
    assert main([a, str(tmp_path / "missing.pt")]) == 2
    _tiny_run(tmp_path / "d", 2, ["--use-torch-distributed-ckpt"])
    assert main([a, str(tmp_path / "d" / "default-exp" / "ckpt_2"), "--distributed"]) == 0


def test_kill_during_save_never_corrupts_latest(tmp_path):
    """A hard kill while ckpt_4 is being written leaves ckpt_2 as `latest` and loadable."""
    code = ("import sys; sys.path.insert(0, %r); "
            "from tests.test_framework import _tiny_run; _tiny_run(%r, 4, ['--verify-checkpoints'])"
            % (str(ROOT), str(tmp_path)))
    env = dict(os.environ, PYRECOVER_FAULT="kill_during_write:ckpt_4", PYRECOVER_FAULT_HOLD_WRITE="ckpt_4")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, timeout=300)
    assert r.returncode == -9, r.stderr.decode()[-2000:]
    from pyrecover_amd.ckpt.core import get_latest_checkpoint
    from pyrecover_amd.ckpt.vanilla import verify_checkpoint

    latest = get_latest_checkpoint(str(tmp_path / "default-exp"))
    assert latest.endswith("ckpt_2.pt")
    assert verify_checkpoint(latest)[0]
    assert not (tmp_path / "default-exp" / "ckpt_4.pt").exists()
    r = _tiny_run(tmp_path, 4, ["--resume-from-checkpoint", "latest", "--verify-checkpoints"])
    assert r["step"] == 4


def test_op_roctx_ranges_toggle():
    """Per-op roctx ranges are switchable at runtime; the trainer turns them on for
    the --profile window."""
    from pyrecover_amd import _ext

    if not _ext.available():
        pytest.skip("native extension not built")
    C = _ext.native()
    was = C.roctx_enabled()
    C.set_roctx(True)
    assert C.roctx_enabled()
    C.set_roctx(False)
    assert not C.roctx_enabled()
    C.set_roctx(was)


def test_time_aware_budgets_async_write_and_drain(monkeypatch):
    """The stop threshold covers the final save and what an in-flight async save still needs:
    the rest of its write (from the engine's byte counters, not from a prior) and its deferred
    whole-file digest."""
    import time as _t

    from pyrecover_amd.ckpt import core as ck
    from pyrecover_amd.timelimit import TimeAwareStopper

    st = TimeAwareStopper(1.0, 10.0, end_time=_t.time() + 1000)
    st.update_iter(1.0)  # steady state: buffer = 5 iter + 1 ckpt
    base = st.threshold
    cost = ck.SaveCostModel(40 * 10**9, inline_md5=True, d2h_gbps=40.0)
    cost.probe_write_bps, cost.probe_md5_bps = 4e9, 1e9
    monkeypatch.setitem(ck.WRITE_STATS, "min_write_bps", 0.0)
    monkeypatch.setitem(ck.WRITE_STATS, "min_inline_bps", 0.0)
    monkeypatch.setattr(ck.Checkpointer, "_instances", {})
    assert cost.final_seconds() == pytest.approx(2.0 + 1.0 + 40.0)
    assert st.set_ckpt_estimate(cost.final_seconds())
    assert st.threshold == pytest.approx(base + 2 * (43.0 - 10.0))  # ckpt + buffer's ckpt term

    class _Eng:
        def busy(self):
            return True

        def progress(self):  # 40 GB periodic save, 16 GB written, deferred digest
            return (40 * 10**9, 16 * 10**9, 0, 2)

        def md5_pending_bytes(self):
            return 0

        def md5_min_bps(self):
            return 0.0

    class _C:
        pending = ck.Job(ckpt=None, path="x", keepalive=None, on_done=None, started=_t.perf_counter())
        engine = _Eng()

    monkeypatch.setattr(ck.Checkpointer, "_instances", {0: _C()})
    drain = cost.drain_seconds(st.ckpt_budget)
    # 24 GB left to write at 4 GB/s = 6 s; its 40 GB digest ends at 6 + 40 = 46 s, before the final
    # save (6 + 43 = 49 s) finishes: the drain is the 6 s write
    assert drain == pytest.approx(6.0)
    st.inflight_drain = drain
    assert st.threshold == pytest.approx(base + 66.0 + 6.0)
    # a digest backlog longer than the final save extends the drain
    monkeypatch.setattr(_Eng, "md5_pending_bytes", lambda self: 20 * 10**9)
    assert cost.drain_seconds(st.ckpt_budget) == pytest.approx(6.0 + 60.0 - 43.0)


def test_save_cost_probe_and_drop_unverified(tmp_path):
    """The startup probes return positive rates (native write path into the checkpoint directory,
    serial MD5), leave no probe file behind, and drop_unverified keeps only verified or newer
    checkpoints."""
    from pyrecover_amd import _ext
    from pyrecover_amd.ckpt import core as ck

    if not _ext.available():
        pytest.skip("native extension not built")
    cost = ck.SaveCostModel(64 << 20, inline_md5=True).probe(tmp_path, write_bytes=128 << 20, md5_bytes=16 << 20)
    assert cost.probe_write_bps > 0 and cost.probe_md5_bps > 0
    assert list(tmp_path.iterdir()) == []
    for n, md5 in ((2, True), (4, False), (6, False)):
        (tmp_path / f"ckpt_{n}.pt").write_bytes(b"x")
        (tmp_path / f"ckpt_{n}.pt.md5parts").write_text("p")
        if md5:
            (tmp_path / f"ckpt_{n}.pt.md5").write_text("0" * 32)
    (tmp_path / "ckpt_5_final.pt").write_bytes(b"x")
    (tmp_path / "ckpt_1.pt").write_bytes(b"x")  # an earlier job's checkpoint, written without a digest
    mine = {str(tmp_path / f"ckpt_{n}.pt") for n in (2, 4, 6)}  # this process deferred their digests
    removed = ck.drop_unverified(tmp_path, str(tmp_path / "ckpt_5_final.pt"), only=mine)
    assert [Path(r).name for r in removed] == ["ckpt_4.pt"]
    assert sorted(p.name for p in tmp_path.glob("*.pt")) == ["ckpt_1.pt", "ckpt_2.pt", "ckpt_5_final.pt",
                                                              "ckpt_6.pt"]
    assert not (tmp_path / "ckpt_4.pt.md5parts").exists()


def test_timeaware_stop_uses_final_save_estimate(tmp_path, monkeypatch):
    """Trainer level: with no save before the stop, the threshold includes the predicted final
    save (here 40 s), so a job with 70 s left stops at step 1 (the reference's 41 s prior would
    keep going)."""
    from pyrecover_amd.ckpt import core as ckcore
    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    monkeypatch.setenv("SLURM_JOB_END_TIME", str(time.time() + 70))
    monkeypatch.setattr(ckcore.SaveCostModel, "final_seconds", lambda self, nbytes=None: 40.0)
    base = ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "2",
            "--training-steps", "20", "--checkpoint-dir", str(tmp_path), "--checkpoint-frequency", "-1",
            "--model-dtype", "fp32", "--num-workers", "0", "--timeaware-checkpointing"]
    r = train(get_args(base))
    assert r["stopped_early"] and r["step"] == 1


def test_loss_csv_log_line_and_metrics_jsonl(tmp_path, caplog):
    """--log-loss-to-csv (reference train.py:143-151, 277-280: <exp>_loss_log.csv with a Step,Loss header
    and one row per step), the reference log-line format (train.py:289-291) and --metrics-jsonl; a
    resumed run appends to the CSV instead of truncating it."""
    import csv
    import json
    import logging

    from pyrecover_amd.cli import get_args
    from pyrecover_amd.trainer import train

    jl = tmp_path / "m.jsonl"
    base = ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "2",
            "--checkpoint-dir", str(tmp_path), "--experiment_name", "e", "--checkpoint-frequency", "3",
            "--model-dtype", "fp32", "--num-workers", "0", "--logging-frequency", "1", "--log-loss-to-csv",
            "--metrics-jsonl", str(jl)]
    with caplog.at_level(logging.INFO):
        train(get_args(base + ["--training-steps", "3"]))
    lines = [r.getMessage() for r in caplog.records if r.getMessage().startswith("Epoch: ")]
    assert len(lines) == 3
    fields = [f.split(":")[0].strip() for f in lines[0].split("|")]
    assert fields[:7] == ["Epoch", "Step", "Loss", "Tokens per second", "Training tokens per second (%)", "MFU (%)",
                          "TFLOPs"]
    train(get_args(base + ["--training-steps", "5", "--resume-from-checkpoint", "latest"]))
    rows = list(csv.reader(open(tmp_path / "e" / "e_loss_log.csv")))
    assert rows[0] == ["Step", "Loss"]
    assert [int(r[0]) for r in rows[1:]] == [1, 2, 3, 4, 5]
    assert all(float(r[1]) == float(r[1]) for r in rows[1:])
    recs = [json.loads(x) for x in open(jl)]
    assert [r["step"] for r in recs][-2:] == [4, 5]


def test_teardown_after_gloo_group():
    """maybe_cleanup_distributed (reference dist_utils.py) on an initialized one-rank gloo group."""
    import torch.distributed as dist

    from pyrecover_amd.parallel import dist as D

    port = 29000 + os.getpid() % 1000
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    assert D.get_world_size() == 1 and D.is_rank0()
    D.maybe_cleanup_distributed()
    assert not dist.is_initialized()
    D.maybe_cleanup_distributed()  # no-op when nothing is initialized


def _micro_model():
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer

    torch.manual_seed(0)
    m = Transformer(get_preset("llama-micro", seq_len=64))
    return m, m.flatten_()


def test_gradient_accumulation_equals_full_batch():
    """--grad-accumulation-steps: two micro-batches written into the same flat gradients (the
    second backward adds) sum to twice the full-batch gradient of the mean loss."""
    m, flat = _micro_model()
    tok = torch.randint(0, m.model_args.vocab_size, (4, 65), generator=torch.Generator().manual_seed(3))
    flat.zero_grad()
    m(tok[:, :-1], labels=tok[:, 1:]).backward()
    full = flat.grad.clone()
    flat.zero_grad()
    for i, sl in enumerate((slice(0, 2), slice(2, 4))):
        if i:
            flat.next_micro_batch()
        m(tok[sl, :-1], labels=tok[sl, 1:]).backward()
    torch.testing.assert_close(flat.grad / 2, full, rtol=1e-4, atol=1e-6)


def test_activation_checkpointing_matches_stored_activations():
    """--activation-checkpointing recomputes each block in backward; loss and gradients are the
    ones of the stored-activation path."""
    m, flat = _micro_model()
    tok = torch.randint(0, m.model_args.vocab_size, (2, 65), generator=torch.Generator().manual_seed(4))
    flat.zero_grad()
    l0 = m(tok[:, :-1], labels=tok[:, 1:])
    l0.backward()
    g0 = flat.grad.clone()
    m.activation_checkpointing = True
    flat.zero_grad()
    l1 = m(tok[:, :-1], labels=tok[:, 1:])
    l1.backward()
    assert torch.equal(l0.detach(), l1.detach())
    torch.testing.assert_close(flat.grad, g0, rtol=1e-5, atol=1e-7)


def test_trainer_grad_accumulation_and_checkpointing_run(tmp_path):
    """The trainer's accumulation loop + recompute path step, checkpoint and resume."""
    r = _tiny_run(tmp_path, 2, ["--grad-accumulation-steps", "2", "--activation-checkpointing"])
    assert r["step"] == 2
    r = _tiny_run(tmp_path, 4, ["--grad-accumulation-steps", "2", "--resume-from-checkpoint", "latest"])
    assert r["step"] == 4


def test_reduction_settings_recorded_pinned_and_compared(tmp_path, caplog, monkeypatch):
    """SURVEY §5.8 determinism contract: every checkpoint records the gradient-reduction settings
    (world size, backend, RCCL algorithm / protocol / channels); a resume under different ones warns;
    PYRECOVER_RCCL_DETERMINISTIC=1 pins ring / Simple / 16 channels where the user set nothing."""
    import logging

    from pyrecover_amd.ckpt import core as ckcore
    from pyrecover_amd.parallel import dist as D

    env = {"PYRECOVER_RCCL_DETERMINISTIC": "1", "NCCL_PROTO": "LL128"}
    pinned = D.pin_rccl_order(env)
    assert env["NCCL_ALGO"] == "Ring" and env["NCCL_PROTO"] == "LL128" and "NCCL_PROTO" not in pinned
    assert env["NCCL_MIN_NCHANNELS"] == env["NCCL_MAX_NCHANNELS"] == "16"
    assert D.pin_rccl_order({}) == {}
    _tiny_run(tmp_path, 2)
    ck = torch.load(tmp_path / "default-exp" / "ckpt_2.pt", weights_only=True)
    red = ck["pyrecover_state"]["reduction"]
    assert red["world_size"] == 1 and "backend" in red
    assert ckcore.warn_reduction_change(ck["pyrecover_state"]) == []
    monkeypatch.setenv("NCCL_ALGO", "Tree")
    with caplog.at_level(logging.WARNING, logger="pyrecover"):
        diffs = ckcore.warn_reduction_change(ck["pyrecover_state"])
    assert diffs and "NCCL_ALGO" in diffs[0] and "gradient-reduction" in caplog.text
