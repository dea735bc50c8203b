"""--compile = HIP-graph capture of the whole training step (pyrecover_amd/graph.py).
A replayed step must produce bit-identical parameters / optimizer state / losses to eager
steps, with the overlapped optimizer and with a changing learning rate (warmup schedule)."""
import pytest
import torch

from pyrecover_amd.config import get_preset
from pyrecover_amd.models.llama import Transformer

pytestmark = pytest.mark.gpu


def _run(cuda, graph: bool, overlap: bool, steps=6, clip=False):
    from pyrecover_amd.graph import StepGraph
    from pyrecover_amd.optim.adamw import FlatAdamW
    from pyrecover_amd.optim.lr import build_lr_scheduler
    from pyrecover_amd.parallel.ddp import GradReducer

    torch.manual_seed(0)
    a = get_preset("llama-tiny", seq_len=256)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(cuda):
        m = Transformer(a)
    torch.set_default_dtype(prev)
    flat = m.flatten_()
    red = GradReducer(flat, bucket_cap_mb=0.5, first_bucket_mb=0.25)
    opt = FlatAdamW(flat, lr=1e-3)
    if overlap:
        opt.enable_overlap(red)
    sched = build_lr_scheduler(opt, 3)  # lr changes every step during warmup
    clip_fn = None
    if clip:
        def clip_fn():
            from pyrecover_amd import _ext
            opt.grad_scale_dev = _ext.native().grad_norm(flat.grad, 0.05, 1.0)[1:2]
    sg = StepGraph(m, opt, red, pre_step=clip_fn) if graph else None
    gen = torch.Generator(device=cuda)
    gen.manual_seed(123)
    losses = []
    for i in range(steps):
        t = torch.randint(0, a.vocab_size, (2, 257), device=cuda, generator=gen)
        x, y = t[:, :-1], t[:, 1:]
        if sg is not None and i >= 2:
            loss = sg.step(x, y)
        else:
            opt.zero_grad()
            loss = m(x, labels=y)
            loss.backward()
            red.finish()
            if clip_fn:
                clip_fn()
            opt.step()
        sched.step()
        losses.append(loss.detach().float().item())
    torch.cuda.synchronize()
    return flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), losses, opt._step, sg


@pytest.mark.parametrize("overlap", [False, True])
def test_graph_step_matches_eager(cuda, overlap):
    p0, m0, v0, l0, s0, _ = _run(cuda, graph=False, overlap=overlap)
    p1, m1, v1, l1, s1, sg = _run(cuda, graph=True, overlap=overlap)
    assert sg.captured and sg.replays == 4
    assert s0 == s1 == 6
    assert l0 == l1
    assert torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1)


def test_graph_step_with_grad_clipping(cuda):
    p0, _, _, l0, _, _ = _run(cuda, graph=False, overlap=False, clip=True)
    p1, _, _, l1, _, _ = _run(cuda, graph=True, overlap=False, clip=True)
    assert l0 == l1 and torch.equal(p0, p1)


def _targs(ckdir, steps, extra=()):
    from pyrecover_amd.cli import get_args

    a = ["--model-preset", "llama-tiny", "--synthetic-data", "--sequence-length", "256", "--batch-size", "2",
         "--training-steps", str(steps), "--checkpoint-dir", str(ckdir), "--experiment_name", "exp",
         "--checkpoint-frequency", "3", "--num-workers", "0", "--logging-frequency", "100",
         "--learning-rate", "1e-3", "--lr-warmup-steps", "2"]
    return get_args(a + list(extra))


def _final(path):
    ck = torch.load(path, weights_only=True)
    return ck["model"], ck["optimizer"]["state"]


def _same(a, b):
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
    for k in a[1]:
        for f in ("exp_avg", "exp_avg_sq", "step"):
            assert torch.equal(a[1][k][f], b[1][k][f]), (k, f)


def test_train_compile_matches_eager_and_resumes_bit_exact(cuda, tmp_path):
    """train.py --compile: same checkpoints as eager training, and a run preempted at step 4
    then resumed (re-captured after its eager warmup steps) ends bit-identical."""
    from pyrecover_amd.trainer import train

    train(_targs(tmp_path / "eager", 6))
    train(_targs(tmp_path / "graph", 6, ["--compile"]))
    _same(_final(tmp_path / "eager" / "exp" / "ckpt_6.pt"), _final(tmp_path / "graph" / "exp" / "ckpt_6.pt"))
    r = train(_targs(tmp_path / "split", 6, ["--compile", "--stop-at-step", "4"]))
    assert r["stopped_early"] and r["step"] == 4
    train(_targs(tmp_path / "split", 6, ["--compile", "--resume-from-checkpoint", "latest"]))
    _same(_final(tmp_path / "graph" / "exp" / "ckpt_6.pt"), _final(tmp_path / "split" / "exp" / "ckpt_6.pt"))
