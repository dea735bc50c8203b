"""Bit-exact resume (SURVEY §7.4 hard part 2): N steps straight == k steps + resume + N-k steps,
tolerance 0, for model weights, AdamW moments, LR schedule and the data stream."""
import os
import zipfile

import pytest
import torch

from pyrecover_amd.cli import get_args
from pyrecover_amd.trainer import train


def _args(ckdir, steps, extra=(), exp="exp", sharded=False, resume=None):
    a = ["--model-preset", "llama-micro", "--synthetic-data", "--sequence-length", "128", "--batch-size", "2",
         "--training-steps", str(steps), "--checkpoint-dir", str(ckdir), "--experiment_name", exp,
         "--checkpoint-frequency", "3", "--model-dtype", "fp32", "--num-workers", "0", "--logging-frequency", "100",
         "--learning-rate", "1e-3", "--lr-warmup-steps", "2", "--verify-checkpoints"]
    if sharded:
        a.append("--use-torch-distributed-ckpt")
    if resume:
        a += ["--resume-from-checkpoint", resume]
    return get_args(a + list(extra))


def _load_final(path, sharded):
    if sharded:
        from pyrecover_amd.ckpt.sharded import read_sharded_state

        st = read_sharded_state(path)
        return st["model"], st["optimizer"], st["lr_scheduler"], st["metadata"]["step"]
    ck = torch.load(path, weights_only=True)
    return ck["model"], ck["optimizer"], ck["lr_scheduler"], ck["step"]


def _assert_same(a, b):
    ma, oa, sa, stepa = a
    mb, ob, sb, stepb = b
    assert stepa == stepb
    assert ma.keys() == mb.keys()
    for k in ma:
        assert torch.equal(ma[k], mb[k]), k
    sa_, sb_ = oa["state"], ob["state"]
    assert {str(k) for k in sa_} == {str(k) for k in sb_}
    for k in sa_:
        kb = k if k in sb_ else str(k)
        for f in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(torch.as_tensor(sa_[k][f]), torch.as_tensor(sb_[kb][f])), (k, f)
    assert sa["last_epoch"] == sb["last_epoch"] and sa["_last_lr"] == sb["_last_lr"]


@pytest.mark.parametrize("sharded", [False, True])
def test_resume_bit_exact(tmp_path, sharded):
    straight = tmp_path / "a"
    train(_args(straight, 6, sharded=sharded))
    split = tmp_path / "b"
    r = train(_args(split, 6, sharded=sharded, extra=["--stop-at-step", "4"]))  # "preempted" at step 4
    assert r["stopped_early"] and r["step"] == 4
    train(_args(split, 6, sharded=sharded, resume="latest"))
    name = "ckpt_6" if sharded else "ckpt_6.pt"
    _assert_same(_load_final(str(straight / "exp" / name), sharded), _load_final(str(split / "exp" / name), sharded))


def test_vanilla_format_is_reference_compatible(tmp_path):
    train(_args(tmp_path, 3))
    p = tmp_path / "exp" / "ckpt_3.pt"
    # md5 sidecar = 32 hex chars of the whole file, no newline (reference checkpoint.py:79-83)
    import hashlib

    md5 = open(str(p) + ".md5").read()
    assert md5 == hashlib.md5(p.read_bytes()).hexdigest() and len(md5) == 32
    assert zipfile.ZipFile(p).testzip() is None  # every CRC32 valid
    ck = torch.load(p, map_location="cpu", mmap=True, weights_only=True)
    assert {"epoch", "step", "model", "optimizer", "lr_scheduler"} <= set(ck)
    keys = list(ck["model"])
    assert keys[0] == "tok_embeddings.weight" and keys[-1] == "output.weight"
    assert "layers.0.attention.wq.weight" in keys and "layers.1.feed_forward.w3.weight" in keys
    assert not any(k.startswith("module.") for k in keys)
    assert "freqs_cis" not in ck["model"]
    opt = ck["optimizer"]
    assert len(opt["state"]) == len(keys) and opt["param_groups"][0]["params"] == list(range(len(keys)))
    assert set(opt["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}
    assert ck["lr_scheduler"]["lr_lambdas"] == [{}]
    # loads into a stock torch.optim.AdamW
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer

    m = Transformer(get_preset("llama-micro", seq_len=128))
    m.load_state_dict(ck["model"])
    o = torch.optim.AdamW(m.parameters(), lr=1e-3)
    o.load_state_dict(ck["optimizer"])


def test_sharded_is_dcp_readable(tmp_path):
    import torch.distributed.checkpoint as dcp

    train(_args(tmp_path, 3, sharded=True))
    d = tmp_path / "exp" / "ckpt_3"
    assert (d / ".metadata").exists() and (d / "__0_0.distcp").exists() and not (d / ".incomplete").exists()
    from pyrecover_amd.ckpt.sharded import read_sharded_state

    ours = read_sharded_state(str(d))
    target = {"model": {k: torch.empty_like(v) for k, v in ours["model"].items()},
              "metadata": {"epoch": 0, "step": 0}}
    dcp.load(target, checkpoint_id=str(d))
    for k, v in ours["model"].items():
        assert torch.equal(target["model"][k], v), k
    assert target["metadata"]["step"] == 3


def test_corrupted_checkpoint_is_refused(tmp_path):
    train(_args(tmp_path, 3))
    p = tmp_path / "exp" / "ckpt_3.pt"
    data = bytearray(p.read_bytes())
    data[len(data) // 2] ^= 0xFF
    p.write_bytes(bytes(data))
    with pytest.raises(RuntimeError, match="Checksum mismatch"):
        train(_args(tmp_path, 6, resume="latest"))
