"""Direct xGMI all-reduce backend (pyrecover_amd/parallel/xgmi.py) with 2 ranks sharing one GPU:
IPC memory + IPC events across processes; the native pull engine (one pull-reduce and one
pull-gather kernel per bucket on one stream, C++ worker).
Checks the all-reduce result against the fp32 sum and that 3 training steps with backend="xgmi"
equal the same steps with the default process-group all-reduce (bit-exact: for 2 ranks the fp32
sum rounded once equals the bf16 sum). Multi-GPU bandwidth is not measured here."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, backend, port, overlap=False):
    out = tmp_path / f"{backend}{'_ov' if overlap else ''}.pt"
    env = dict(os.environ, PYRECOVER_LOCAL_DEVICE="0", PYRECOVER_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "dist_workers", "xgmi_worker.py"),
           "--backend", backend, "--out", str(out)] + (["--overlap"] if overlap else [])
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    return torch.load(out, weights_only=True)


def test_xgmi_allreduce_matches_process_group(cuda, tmp_path):
    port = 29531
    a = _run(tmp_path, "rccl", port)
    b = _run(tmp_path, "xgmi", port + 1)
    assert b["direct_err"] == 0.0 and a["direct_err"] == 0.0
    assert torch.equal(a["params"], b["params"])
    c = _run(tmp_path, "xgmi", port + 2, overlap=True)
    assert torch.equal(a["params"], c["params"])


def test_rccl_process_group_with_high_priority_stream(cuda):
    """The RCCL process-group options used by parallel/dist.py are accepted by this build."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dist_workers", "rccl_single.py"), "29541"],
                       env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "rccl ok" in r.stdout, (r.stdout + r.stderr)[-4000:]
