"""Asynchronous checkpoint snapshot on the GPU: the two-hop (HBM bounce buffer, then D2H) snapshot
fences the next update only on its device-to-device copy; what lands on disk is the state at save
time even when the parameters and moments are overwritten right after the fence."""
import pytest
import torch

from pyrecover_amd.config import get_preset
from pyrecover_amd.models.llama import Transformer

pytestmark = pytest.mark.gpu


def _setup(cuda):
    from pyrecover_amd.optim.adamw import FlatAdamW

    torch.manual_seed(0)
    cfg = get_preset("llama-tiny", seq_len=128)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(cuda):
        m = Transformer(cfg)
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    opt = FlatAdamW(flat, lr=1e-3)
    t = torch.randint(0, cfg.vocab_size, (2, 129), device=cuda)
    opt.zero_grad()
    m(t[:, :-1], labels=t[:, 1:]).backward()
    opt.step()
    return m, flat, opt


@pytest.mark.parametrize("mode", ["two_hop", "direct", "no_room"])
def test_async_snapshot_is_the_state_at_save_time(cuda, tmp_path, monkeypatch, mode):
    from pyrecover_amd.ckpt import core
    from pyrecover_amd.ckpt.vanilla import save_ckpt_vanilla

    if mode == "direct":
        monkeypatch.setenv("PYRECOVER_CKPT_HBM", "0")
    if mode == "no_room":  # free HBM below the reserve: falls back to the direct D2H snapshot
        monkeypatch.setenv("PYRECOVER_CKPT_HBM_RESERVE_GB", "1000000")
    m, flat, opt = _setup(cuda)
    ck = core.Checkpointer.get(flat.data.device)
    monkeypatch.setattr(ck, "_hbm", None)
    want_p = flat.data.clone()
    want_v = opt.exp_avg_sq.clone()
    p = tmp_path / "ckpt_1.pt"
    save_ckpt_vanilla(m, opt, None, None, 1, 1, str(p), max_keep=0, verify=False, async_save=True)
    assert ck.engine.last_two_hop() == (mode == "two_hop")
    core.fence_all()  # what the optimizer does before its next update
    flat.data.fill_(7.0)  # overwrite the live buffers at once (the next update)
    opt.exp_avg_sq.fill_(3.0)
    core.wait_all()
    sd = torch.load(p, weights_only=True, map_location="cpu")
    for n, prm in m.named_parameters():
        o = flat.param_offset[id(prm)]
        got = sd["model"][n].to(cuda).reshape(-1)
        assert torch.equal(got, want_p[o:o + prm.numel()]), n
    for i, st in sd["optimizer"]["state"].items():
        prm = opt.param_groups[0]["params"][int(i)]
        o = flat.param_offset[id(prm)]
        assert torch.equal(st["exp_avg_sq"].to(cuda).reshape(-1), want_v[o:o + prm.numel()]), i
