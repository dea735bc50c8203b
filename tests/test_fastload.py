"""Native resume path (pyrecover_amd.ckpt.fastload + _C.CkptReader) on CPU:

* the native reader places exactly the bytes torch.load sees (vanilla + sharded), bit for bit;
* the writer's ``.md5parts`` sidecar is the MD5 of every 256 MiB segment (hashlib oracle) and the
  whole-file ``.md5`` is unchanged; corruption is caught through either sidecar;
* world 2 (gloo): every rank reads about half of the bytes and the flat buffers are completed by
  an all-gather, bit-exact.
"""
import hashlib
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from pyrecover_amd import _ext
from pyrecover_amd.ckpt import core, fastload
from pyrecover_amd.ckpt.sharded import MANIFEST, load_ckpt_distributed, save_ckpt_distributed
from pyrecover_amd.ckpt.vanilla import load_ckpt_vanilla, save_ckpt_vanilla
from pyrecover_amd.config import get_preset
from pyrecover_amd.models.llama import Transformer
from pyrecover_amd.optim.adamw import FlatAdamW
from pyrecover_amd.optim.lr import build_lr_scheduler

pytestmark = pytest.mark.skipif(not _ext.available(), reason="native extension not built")


def _build(seed=0, dtype=torch.float32):
    torch.manual_seed(seed)
    m = Transformer(get_preset("llama-micro", seq_len=64)).to(dtype)
    flat = m.flatten_()
    opt = FlatAdamW(flat, lr=1e-3)
    return m, flat, opt, build_lr_scheduler(opt, 4)


def _train(m, opt, sched, steps=2):
    g = torch.Generator().manual_seed(5)
    for _ in range(steps):
        t = torch.randint(0, m.vocab_size, (2, 65), generator=g)
        opt.zero_grad()
        m(t[:, :-1], labels=t[:, 1:]).backward()
        opt.step()
        sched.step()


def _same(a_m, a_opt, b_m, b_opt):
    assert torch.equal(a_m.flat.data, b_m.flat.data)
    assert torch.equal(a_opt.exp_avg, b_opt.exp_avg) and torch.equal(a_opt.exp_avg_sq, b_opt.exp_avg_sq)
    assert a_opt._step == b_opt._step


def test_native_reader_matches_torch_load(tmp_path):
    m, flat, opt, sched = _build()
    _train(m, opt, sched)
    p = str(tmp_path / "ckpt_2.pt")
    save_ckpt_vanilla(m, opt, sched, None, 2, 1, p, max_keep=0, verify=True)
    # plan: every parameter and moment is a native item, nothing left to torch
    m2, _, opt2, sched2 = _build(seed=1)
    ckpt, plan = fastload.plan_vanilla(p, m2, opt2)
    assert not plan.fallback and plan.opt_tensors
    assert plan.nbytes() == 3 * flat.data.numel() * flat.data.element_size()
    stats = fastload.execute(plan, fastload.flat_buffers(m2, opt2), True, fastload.read_md5parts(p), p)
    fastload.finish_state(m2, opt2, sched2, None, ckpt, plan)
    assert stats["verified"] == "md5parts"
    _same(m, opt, m2, opt2)
    # the same bytes torch.load reads
    ref = torch.load(p, weights_only=True)
    for k, v in m2.state_dict().items():
        assert torch.equal(v, ref["model"][k]), k
    assert sched2.state_dict()["last_epoch"] == sched.state_dict()["last_epoch"]


def test_md5parts_sidecar_and_corruption(tmp_path):
    m, flat, opt, sched = _build()
    _train(m, opt, sched, 1)
    p = str(tmp_path / "ckpt_1.pt")
    save_ckpt_vanilla(m, opt, sched, None, 1, 1, p, max_keep=0, verify=True)
    data = open(p, "rb").read()
    # the whole-file .md5 is a deferred background digest: it exists once flushed (and before
    # the staging pool is reused / at exit); .md5parts exists when the save returns
    assert os.path.exists(p + ".md5parts")
    core.flush_all()
    assert open(p + ".md5").read() == hashlib.md5(data).hexdigest()
    seg, total, md5s = fastload.read_md5parts(p)
    assert total == len(data) and seg == _ext.native().MD5PARTS_SEGMENT_BYTES
    assert md5s == [hashlib.md5(data[i:i + seg]).hexdigest() for i in range(0, len(data), seg)]
    # a flipped payload byte is caught by the parallel segment check...
    b = bytearray(data)
    b[len(b) // 2] ^= 0xFF
    open(p, "wb").write(bytes(b))
    m2, _, opt2, sched2 = _build(seed=1)
    with pytest.raises(RuntimeError, match="Checksum mismatch"):
        load_ckpt_vanilla(m2, opt2, sched2, None, p, verify=True)
    # ... and by the whole-file .md5 when there is no .md5parts (reference-written checkpoints)
    os.remove(p + ".md5parts")
    with pytest.raises(RuntimeError, match="Checksum mismatch"):
        load_ckpt_vanilla(m2, opt2, sched2, None, p, verify=True)
    open(p, "wb").write(data)
    load_ckpt_vanilla(m2, opt2, sched2, None, p, verify=True)
    _same(m, opt, m2, opt2)


def test_reference_layout_checkpoint_takes_native_path(tmp_path):
    """A plain torch.save of the reference's dict (per-tensor storages, no md5parts) is planned
    natively too: offsets come from the zip directory of the mmap'ed archive."""
    m, flat, opt, sched = _build()
    _train(m, opt, sched, 1)
    p = str(tmp_path / "ref.pt")
    torch.save({"epoch": 1, "step": 1, "model": {k: v.clone() for k, v in m.state_dict().items()},
                "optimizer": opt.state_dict(), "lr_scheduler": sched.state_dict()}, p)
    m2, _, opt2, sched2 = _build(seed=1)
    ckpt, plan = fastload.plan_vanilla(p, m2, opt2)
    assert not plan.fallback and plan.opt_tensors
    fastload.execute(plan, fastload.flat_buffers(m2, opt2))
    fastload.finish_state(m2, opt2, sched2, None, ckpt, plan)
    _same(m, opt, m2, opt2)


def test_sharded_manifest_fast_path(tmp_path):
    m, flat, opt, sched = _build()
    _train(m, opt, sched)
    d = str(tmp_path / "ckpt_2")
    save_ckpt_distributed(m, opt, sched, None, 2, 1, d, max_keep=0)
    import json

    man = json.loads(open(os.path.join(d, MANIFEST)).read())
    assert all("data_offset" in e for k, e in man.items() if k.startswith("model."))
    m2, _, opt2, sched2 = _build(seed=1)
    ckpt, plan = fastload.plan_sharded(d, m2, opt2)
    assert not plan.fallback and plan.opt_tensors and plan.nbytes() == 3 * flat.state_bytes() // 3 * 3
    load_ckpt_distributed(m2, opt2, sched2, None, d)
    _same(m, opt, m2, opt2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _w2(rank, world, port, path, kind, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    m2, _, opt2, sched2 = _build(seed=1 + rank)
    if kind == "vanilla":
        ckpt, plan = fastload.plan_vanilla(path, m2, opt2)
        stats = fastload.execute(plan, fastload.flat_buffers(m2, opt2), True, fastload.read_md5parts(path), path,
                                 is_distributed=True)
    else:
        ckpt, plan = fastload.plan_sharded(path, m2, opt2)
        stats = fastload.execute(plan, fastload.flat_buffers(m2, opt2), is_distributed=True)
    fastload.finish_state(m2, opt2, sched2, None, ckpt, plan)
    torch.save({"data": m2.flat.data, "m": opt2.exp_avg, "v": opt2.exp_avg_sq, "step": opt2._step,
                "item_bytes": stats["item_bytes"]}, os.path.join(out, f"r{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["vanilla", "sharded"])
def test_two_ranks_read_half_and_allgather(tmp_path, kind):
    m, flat, opt, sched = _build()
    _train(m, opt, sched)
    path = str(tmp_path / ("ckpt_2.pt" if kind == "vanilla" else "ckpt_2"))
    if kind == "vanilla":
        save_ckpt_vanilla(m, opt, sched, None, 2, 1, path, max_keep=0, verify=True)
    else:
        save_ckpt_distributed(m, opt, sched, None, 2, 1, path, max_keep=0)
    mp.spawn(_w2, args=(2, _free_port(), path, kind, str(tmp_path)), nprocs=2, join=True)
    total = 3 * flat.data.numel() * flat.data.element_size()
    for r in range(2):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        assert torch.equal(got["data"], flat.data) and torch.equal(got["m"], opt.exp_avg)
        assert torch.equal(got["v"], opt.exp_avg_sq) and got["step"] == opt._step
        # each rank places its half of every flat buffer (plus a < world-byte tail) from the file
        assert total // 2 <= got["item_bytes"] <= total // 2 + 3 * 2


_EINVAL_SCRIPT = r"""
import json, sys, torch
sys.path.insert(0, {root!r})
from pyrecover_amd.ckpt import core
from pyrecover_amd.ckpt.vanilla import save_ckpt_vanilla, load_ckpt_vanilla
from pyrecover_amd.config import get_preset
from pyrecover_amd.models.llama import Transformer
from pyrecover_amd.optim.adamw import FlatAdamW
torch.manual_seed(0)
m = Transformer(get_preset("llama-micro", seq_len=64)); flat = m.flatten_(); opt = FlatAdamW(flat, lr=1e-3)
save_ckpt_vanilla(m, opt, step=3, epoch=1, checkpoint_path={path!r}, verify=True)
direct = core.WRITE_STATS["last"]["direct"]
ref = torch.load({path!r}, weights_only=True)
m2 = Transformer(get_preset("llama-micro", seq_len=64)); flat2 = m2.flatten_(); opt2 = FlatAdamW(flat2, lr=1e-3)
load_ckpt_vanilla(m2, opt2, checkpoint_path={path!r}, verify=True)
ok = torch.equal(flat.data, flat2.data) and all(torch.equal(ref["model"][k], v) for k, v in m.state_dict().items())
print(json.dumps({{"direct": direct, "ok": ok}}))
"""


@pytest.mark.parametrize("inject", [False, True])
def test_direct_write_refused_falls_back_to_buffered(tmp_path, inject):
    """A filesystem that accepts the O_DIRECT open but refuses the aligned pwrite (EINVAL) must not
    fail the save: the writer switches to buffered writes (PYRECOVER_FAULT_DIRECT_EINVAL injects
    the refusal on the first direct write)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = str(tmp_path / "ckpt_3.pt")
    env = dict(os.environ, PYRECOVER_FAULT_DIRECT_EINVAL="1" if inject else "0", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-c", _EINVAL_SCRIPT.format(root=root, path=path)], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"]
    with open(path, "rb") as f:
        assert hashlib.md5(f.read()).hexdigest() == open(path + ".md5").read()
    if inject:
        assert out["direct"] is False
