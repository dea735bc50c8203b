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
