#!/usr/bin/env python
"""Per-step kernel breakdown of a rocprofv3 --kernel-trace CSV of bench.py: splits the trace into
steps at the embedding-forward kernel, keeps the last N steps, and reports per-kernel (and per
GEMM grid shape) device time per step, the stream split and the step's idle time.

  python tools/trace_summary.py gpurun_out/prof/run_kernel_trace.csv [--steps 2] [--by-grid]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--by-grid", action="store_true", help="split GEMM kernels by grid size")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "embed_fwd_kernel" in r["Kernel_Name"]]
    if len(starts) < a.steps + 1:
        raise SystemExit(f"need {a.steps + 1} step markers, found {len(starts)}")
    lo, hi = starts[-a.steps - 1], starts[-1]
    sel = rows[lo:hi]
    t0, t1 = int(rows[lo]["Start_Timestamp"]), int(rows[hi]["Start_Timestamp"])
    wall = (t1 - t0) / 1e6 / a.steps
    per = collections.defaultdict(lambda: [0.0, 0])
    per_stream = collections.defaultdict(float)
    busy = []
    for r in sel:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        name = r["Kernel_Name"]
        gemm = name.startswith("Custom_Cijk") or "Cijk" in name
        key = name[:90]
        if gemm:
            key = "GEMM " + (f"grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']} " if a.by_grid else "") + name.split("_MT")[1][:20] if "_MT" in name else name[:60]
        elif a.by_grid and ("wgrad" in name or "gemm_nt" in name or "attn" in name):
            key = f"{name[:60]} grid {r['Grid_Size_X']}"
        per[key][0] += d / a.steps
        per[key][1] += 1
        per_stream[r["Queue_Id"]] += d / a.steps
        busy.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    busy.sort()
    cov, cur_s, cur_e = 0, None, None
    for s, e in busy:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                cov += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    cov += cur_e - cur_s
    gemm_ms = sum(v[0] for k, v in per.items() if k.startswith("GEMM"))
    print(f"step wall {wall:.1f} ms; device busy (any queue) {cov / 1e6 / a.steps:.1f} ms; "
          f"GEMM {gemm_ms:.1f} ms; per queue {dict((k, round(v, 1)) for k, v in per_stream.items())}")
    print("ms_per_step,calls_per_step,kernel")
    for k, (ms, n) in sorted(per.items(), key=lambda x: -x[1][0])[:a.top]:
        print(f"{ms:.2f},{n // a.steps},{k}")


if __name__ == "__main__":
    main()
