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


def test_baseline_config1_gpt2_small_fp32_cpu(tmp_path):
    """BASELINE.json config 1: GPT-2-small-shape fp32, seq 128, world_size 1 on CPU, save + resume
    through the pyrecover.checkpoint API (reference-compatible package)."""
    import pyrecover
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler

    def build():
        torch.manual_seed(0)
        m = Transformer(get_preset("gpt2-small", seq_len=128))
        flat = m.flatten_()
        o = FlatAdamW(flat, lr=1e-3)
        return m, o, build_lr_scheduler(o, 10)

    tok = torch.randint(0, 50304, (2, 129), generator=torch.Generator().manual_seed(1))
    m, o, s = build()
    for _ in range(2):
        o.zero_grad()
        m(tok[:, :-1], labels=tok[:, 1:]).backward()
        o.step()
        s.step()
    p = str(tmp_path / "ckpt_2.pt")
    pyrecover.save_ckpt_vanilla(m, o, s, None, 2, 1, p, max_keep=3, verify=True)
    m2, o2, s2 = build()
    epoch, step = pyrecover.load_ckpt_vanilla(m2, o2, s2, None, "latest", experiment_dir=str(tmp_path), verify=True)
    assert (epoch, step) == (1, 2)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    assert torch.equal(o.exp_avg_sq, o2.exp_avg_sq) and s.state_dict() == s2.state_dict()


def test_imports_reference_dcp_checkpoint(tmp_path):
    """A checkpoint written the way the reference writes its sharded format (dcp.save of the
    nn.Module, the torch.optim.AdamW and the LambdaLR objects, reference checkpoint.py:252-274)
    loads into the flat model / FlatAdamW with identical weights and moments."""
    import torch.distributed.checkpoint as dcp

    from pyrecover_amd.ckpt.sharded import load_ckpt_distributed
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler

    torch.manual_seed(0)
    a = get_preset("llama-micro", seq_len=64)
    ref_model = Transformer(a)
    ref_opt = torch.optim.AdamW(ref_model.parameters(), lr=1e-3)
    ref_sched = build_lr_scheduler(ref_opt, 2)
    tok = torch.randint(0, a.vocab_size, (2, 65))
    ref_opt.zero_grad()
    ref_model(tok[:, :-1], labels=tok[:, 1:]).backward()
    ref_opt.step()
    ref_sched.step()
    path = tmp_path / "exp" / "ckpt_1"
    path.parent.mkdir(parents=True)
    dcp.save({"model": ref_model, "optimizer": ref_opt, "metadata": {"epoch": 1, "step": 1},
              "lr_scheduler": ref_sched}, checkpoint_id=str(path), storage_writer=dcp.FileSystemWriter(str(path)))

    torch.manual_seed(1)
    m = Transformer(a)
    flat = m.flatten_()
    opt = FlatAdamW(flat, lr=1e-3)
    sched = build_lr_scheduler(opt, 2)
    epoch, step = load_ckpt_distributed(m, opt, sched, None, str(path))
    assert (epoch, step) == (1, 1)
    ref_sd = ref_model.state_dict()
    for k, v in m.state_dict().items():
        assert torch.equal(v, ref_sd[k]), k
    ref_st = ref_opt.state_dict()["state"]
    for i, p in enumerate(m.parameters()):
        assert torch.equal(opt.state[p]["exp_avg"], ref_st[i]["exp_avg"])
        assert torch.equal(opt.state[p]["exp_avg_sq"], ref_st[i]["exp_avg_sq"])
    assert sched.last_epoch == ref_sched.last_epoch


def test_imports_reference_vanilla_checkpoint(tmp_path):
    """A `.pt` written the way the reference writes it (torch.save of model/optimizer/scheduler
    state dicts, reference checkpoint.py:58-84) resumes into the flat model / FlatAdamW with the
    same weights, moments and schedule; our own vanilla save of the same state has the same
    optimizer index -> tensor mapping."""
    from pyrecover_amd.ckpt.vanilla import load_ckpt_vanilla, save_ckpt_vanilla
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler

    torch.manual_seed(0)
    a = get_preset("llama-micro", seq_len=64)
    ref_model = Transformer(a)
    ref_opt = torch.optim.AdamW(ref_model.parameters(), lr=1e-3)
    ref_sched = build_lr_scheduler(ref_opt, 2)
    tok = torch.randint(0, a.vocab_size, (2, 65))
    ref_opt.zero_grad()
    ref_model(tok[:, :-1], labels=tok[:, 1:]).backward()
    ref_opt.step()
    ref_sched.step()
    p = tmp_path / "exp" / "ckpt_1.pt"
    p.parent.mkdir(parents=True)
    torch.save({"epoch": 1, "step": 1, "model": ref_model.state_dict(), "optimizer": ref_opt.state_dict(),
                "lr_scheduler": ref_sched.state_dict()}, p)

    m = Transformer(a)
    flat = m.flatten_()
    opt = FlatAdamW(flat, lr=1e-3)
    sched = build_lr_scheduler(opt, 2)
    assert load_ckpt_vanilla(m, opt, sched, None, str(p), verify=False) == (1, 1)
    ref_st = ref_opt.state_dict()["state"]
    for i, q in enumerate(m.parameters()):
        assert torch.equal(q, dict(ref_model.named_parameters())[list(dict(m.named_parameters()))[i]])
        assert torch.equal(opt.state[q]["exp_avg"], ref_st[i]["exp_avg"])
    # round trip through our writer keeps the reference's index -> tensor mapping
    p2 = tmp_path / "exp" / "ckpt_2.pt"
    save_ckpt_vanilla(m, opt, sched, None, 2, 1, str(p2), max_keep=0, verify=False)
    ours = torch.load(p2, weights_only=True)["optimizer"]["state"]
    for i in ref_st:
        assert torch.equal(ours[i]["exp_avg_sq"], ref_st[i]["exp_avg_sq"]), i


def test_async_sharded_checkpoint_survives_poll_and_next_save(tmp_path):
    """Regression (advisor r1, high): an async sharded save whose write is collected by poll_all()
    or by the next save must still get its full .metadata, and must be resumable."""
    import time

    from pyrecover_amd.ckpt import core
    from pyrecover_amd.ckpt.sharded import load_ckpt_distributed, read_sharded_state, save_ckpt_distributed
    from pyrecover_amd.config import get_preset
    from pyrecover_amd.models.llama import Transformer
    from pyrecover_amd.optim.adamw import FlatAdamW

    torch.manual_seed(0)
    cfg = get_preset("llama-micro", seq_len=64)
    model = Transformer(cfg)
    opt = FlatAdamW(model.flatten_(), lr=1e-3)
    x = torch.randint(0, cfg.vocab_size, (2, 65))

    def step():
        opt.zero_grad()
        model(x[:, :-1], labels=x[:, 1:]).backward()
        opt.step()

    step()
    d10, d20 = tmp_path / "ckpt_10", tmp_path / "ckpt_20"
    save_ckpt_distributed(model, opt, step=10, epoch=0, checkpoint_path=str(d10), async_save=True)
    snap = {k: v.detach().clone() for k, v in model.state_dict().items()}
    for _ in range(50):  # let the background write finish, then collect it the way the trainer does
        if not any(c.busy() for c in core.Checkpointer._instances.values()):
            break
        time.sleep(0.05)
    core.poll_all()
    step()
    save_ckpt_distributed(model, opt, step=20, epoch=0, checkpoint_path=str(d20), async_save=False)
    for d in (d10, d20):
        assert (d / ".metadata").exists() and not (d / ".incomplete").exists()
        st = read_sharded_state(str(d))
        assert st["model"].keys() == model.state_dict().keys(), d
    fresh = Transformer(cfg)
    fopt = FlatAdamW(fresh.flatten_(), lr=1e-3)
    epoch, s = load_ckpt_distributed(fresh, fopt, checkpoint_path=str(d10))
    assert s == 10
    for k, v in fresh.state_dict().items():
        assert torch.equal(v, snap[k]), k


@pytest.mark.parametrize("sharded", [False, True])
def test_resume_bit_exact_fp32_master_weights(tmp_path, sharded):
    """--master-weights fp32 (optional): bf16 model, fp32 master and moments; the master
    is checkpointed next to the moments and a resumed run is bit-identical, master included."""
    extra = ["--model-dtype", "bf16", "--master-weights", "fp32"]
    straight = tmp_path / "a"
    train(_args(straight, 6, extra, sharded=sharded))
    split = tmp_path / "b"
    r = train(_args(split, 6, extra + ["--stop-at-step", "4"], sharded=sharded))
    assert r["stopped_early"] and r["step"] == 4
    train(_args(split, 6, extra, sharded=sharded, resume="latest"))
    name = "ckpt_6" if sharded else "ckpt_6.pt"
    a = _load_final(str(straight / "exp" / name), sharded)
    b = _load_final(str(split / "exp" / name), sharded)
    _assert_same(a, b)
    sa_, sb_ = a[1]["state"], b[1]["state"]
    for k in sa_:
        kb = k if k in sb_ else str(k)
        ma, mb = sa_[k]["master_param"], sb_[kb]["master_param"]
        assert ma.dtype == torch.float32 and torch.equal(ma, mb), k
        assert sa_[k]["exp_avg"].dtype == torch.float32
    # the model's bf16 parameters are the master rounded
    sid = next(iter(sa_))
    assert any(torch.equal(v.float(), sa_[sid]["master_param"].to(torch.bfloat16).float())
               for v in a[0].values() if v.shape == sa_[sid]["master_param"].shape)


def test_fp32_master_resumes_from_pure_bf16_checkpoint(tmp_path):
    """A pure-bf16 checkpoint (no master in the optimizer state, e.g. the reference's) resumed with
    --master-weights fp32: the master starts from the loaded parameters, the moments are widened."""
    ck = tmp_path / "c"
    train(_args(ck, 3, ["--model-dtype", "bf16"]))
    st3 = torch.load(str(ck / "exp" / "ckpt_3.pt"), weights_only=True)["optimizer"]["state"]
    assert all("master_param" not in v for v in st3.values())
    r = train(_args(ck, 6, ["--model-dtype", "bf16", "--master-weights", "fp32"], resume="latest"))
    assert r["step"] == 6
    st6 = torch.load(str(ck / "exp" / "ckpt_6.pt"), weights_only=True)["optimizer"]["state"]
    for v in st6.values():
        assert v["master_param"].dtype == torch.float32 and v["exp_avg"].dtype == torch.float32
