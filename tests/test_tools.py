"""CPU tests of the measurement tools whose output the README quotes: the exposed-communication
model of tools/comm_predict.py and the per-step kernel breakdown of tools/trace_summary.py."""
import csv
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_comm_predict_simulate_in_order_stream():
    from comm_predict import simulate

    gb = 1e9
    # two 1 GB buckets, 8 ranks, 100 GB/s bus bandwidth, no latency: each all-reduce takes
    # 2 * 7/8 * 1 GB / 100 GB/s = 17.5 ms; the second waits for the first (in-order stream)
    exposed, ends, _ = simulate(ready=[10.0, 12.0], bwd_end=20.0, nbytes=[gb, gb], world=8, busbw_gbps=100.0,
                                latency_us=0.0)
    assert ends == pytest.approx([27.5, 45.0])
    assert exposed == pytest.approx(25.0)
    # a bucket that is ready after the previous one finished starts at its ready time
    exposed, ends, _ = simulate([0.0, 50.0], 60.0, [gb, gb], 8, 100.0, 0.0)
    assert ends == pytest.approx([17.5, 67.5])
    assert exposed == pytest.approx(7.5)
    # fully hidden: nothing exposed; per-collective latency is added to every bucket
    exposed, ends, _ = simulate([0.0], 100.0, [gb], 8, 100.0, 1000.0)
    assert ends == pytest.approx([18.5]) and exposed == 0.0


def test_comm_predict_models_updates_and_sharding():
    """The AdamW update of a bucket waits for its reduction (in-order side stream) and can be what
    is exposed; ZeRO-1 halves the reduction's bus bytes, divides the update by N and adds the
    parameter all-gather on the same FIFO stream (RS_0, RS_1, AG_0, AG_1)."""
    from comm_predict import simulate

    gb = 1e9
    # all-reduce 17.5 ms each; updates of 10 ms each (20 ms for the whole model)
    exp, ends, upd = simulate([10.0, 12.0], 20.0, [gb, gb], 8, 100.0, 0.0, adamw_ms=20.0)
    assert ends == pytest.approx([27.5, 45.0]) and upd == pytest.approx([37.5, 55.0]) and exp == pytest.approx(35.0)
    # one GPU: no communication, the updates alone (what the measured 1-GPU step already contains)
    exp1, _, upd1 = simulate([10.0, 12.0], 20.0, [gb, gb], 1, 1.0, 0.0, adamw_ms=20.0)
    assert upd1 == pytest.approx([20.0, 30.0]) and exp1 == pytest.approx(10.0)
    # ZeRO-1: RS 8.75 ms, update 1.25 ms, AG 8.75 ms (behind its update)
    exp, ends, upd = simulate([10.0, 12.0], 20.0, [gb, gb], 8, 100.0, 0.0, adamw_ms=20.0, mode="shard")
    # RS_0 10 -> 18.75, u_0 -> 20.0; RS_1 18.75 -> 27.5, u_1 -> 28.75; AG_0 27.5 -> 36.25; AG_1 -> 45.0
    assert ends == pytest.approx([18.75, 27.5, 36.25, 45.0]) and upd == pytest.approx([20.0, 28.75])
    assert exp == pytest.approx(25.0)
    # sparse embedding exchange: the last bucket becomes a small all-gather
    exp_s, ends_s, _ = simulate([10.0, 12.0], 20.0, [gb, gb], 8, 100.0, 0.0, adamw_ms=20.0,
                                sparse_bytes=0.1 * gb)
    assert ends_s[-1] == pytest.approx(27.5 + 0.875) and exp_s < 35.0


def _write_trace(path, rows):
    cols = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Grid_Size_X", "Grid_Size_Y",
            "Grid_Size_Z"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        for r in rows:
            w.writerow(dict(zip(cols, r)))


def test_trace_summary_steps_and_grid_split(tmp_path):
    ms = 1_000_000  # ns
    rows = []
    t = 0
    for step in range(3):
        rows.append(("pra::embed_fwd_kernel<bf16>", t, t + 1 * ms, 1, 256, 1, 1))
        rows.append(("Cijk_Ailk_Bljk_BBS_BH_MT256x256x64_MI16x16x1_foo", t + 1 * ms, t + 5 * ms, 1, 65536, 1, 1))
        rows.append(("Cijk_Ailk_Bljk_BBS_BH_MT256x256x64_MI16x16x1_foo", t + 5 * ms, t + 7 * ms, 1, 1024, 1, 1))
        rows.append(("pra::wg::wgrad16_kernel<bf16>", t + 7 * ms, t + 9 * ms, 1, 2048, 1, 1))
        rows.append(("pra::adamw_t_kernel<bf16>", t + 7 * ms, t + 8 * ms, 2, 4096, 1, 1))
        t += 10 * ms
    rows.append(("pra::embed_fwd_kernel<bf16>", t, t + ms, 1, 256, 1, 1))
    trace = tmp_path / "t_kernel_trace.csv"
    _write_trace(trace, rows)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), str(trace), "--steps", "2"],
                         capture_output=True, text=True, check=True).stdout
    head = out.splitlines()[0]
    assert "step wall 10.0 ms" in head and "GEMM 6.0 ms" in head
    assert "'2': 1.0" in head  # the side queue's AdamW time per step
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), str(trace), "--steps", "2",
                          "--by-grid"], capture_output=True, text=True, check=True).stdout
    lines = out.splitlines()
    assert any(line.startswith("4.00,1,GEMM grid 65536x1x1") for line in lines)
    assert any(line.startswith("2.00,1,GEMM grid 1024x1x1") for line in lines)
    assert any("wgrad16_kernel" in line and "grid 2048" in line for line in lines)
    # --overlap: the wgrad call (7-9 ms) runs beside the update (7-8 ms) for half its time, so it
    # counts as alone; --by-predecessor tells the two GEMM grids apart by the kernel before them
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_summary.py"), str(trace), "--steps", "2",
                          "--overlap", "--by-predecessor"], capture_output=True, text=True, check=True).stdout
    assert "calls beside the update" in out
    wl = [line for line in out.splitlines() if line.startswith("pra::wg::wgrad16_kernel")]
    assert wl and wl[-1].split(", ")[1] == "2" and wl[-1].split(", ")[3] == "0"
    pred = [line for line in out.splitlines() if line.startswith(("65536, ", "1024, "))]
    assert any(line.startswith("65536, pra::embed_fwd_kernel<bf16>, 1, 4000.0") for line in pred), pred
    assert any(line.startswith("1024, GEMM grid 65536, 1, 2000.0") for line in pred), pred
