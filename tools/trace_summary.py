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
    ap.add_argument("--by-predecessor", action="store_true",
                    help="library GEMMs grouped by grid and the main-queue kernel before them (tells apart GEMMs "
                         "of one grid size, e.g. the O projection from W2)")
    ap.add_argument("--overlap", action="store_true",
                    help="per kernel: mean duration of the calls that ran beside the AdamW update vs alone")
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
    if a.overlap:
        overlap_report(sel, a)
    if a.by_predecessor:
        predecessor_report(sel, a)


def predecessor_report(sel, a):
    main_q = collections.Counter(r["Queue_Id"] for r in sel).most_common(1)[0][0]
    seq = [r for r in sel if r["Queue_Id"] == main_q]
    acc = collections.defaultdict(lambda: [0, 0.0])
    for prev, r in zip(seq, seq[1:]):
        if "Cijk" not in r["Kernel_Name"]:
            continue
        pn = prev["Kernel_Name"]
        pn = ("GEMM grid " + prev["Grid_Size_X"]) if "Cijk" in pn else pn.split("(")[0][-60:]
        key = (r["Grid_Size_X"], pn)
        acc[key][0] += 1
        acc[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print("\nGEMM grid, previous main-queue kernel, calls per step, mean us")
    for (g, pn), (n, t) in sorted(acc.items(), key=lambda x: -x[1][1]):
        print(f"{g}, {pn}, {n // a.steps}, {t / n:.1f}")


def overlap_report(sel, a):
    """Calls of each non-update kernel split by whether an AdamW kernel ran during most of them."""
    upd = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in sel if "adamw" in r["Kernel_Name"])
    merged = []
    for s, e in upd:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    import bisect

    starts = [m[0] for m in merged]

    def covered(s, e):
        i = max(bisect.bisect_right(starts, s) - 1, 0)
        c = 0
        while i < len(merged) and merged[i][0] < e:
            c += max(0, min(e, merged[i][1]) - max(s, merged[i][0]))
            i += 1
        return c

    acc = collections.defaultdict(lambda: [0, 0.0, 0, 0.0])
    for r in sel:
        name = r["Kernel_Name"]
        if "adamw" in name:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        key = ("GEMM grid " + r["Grid_Size_X"]) if "Cijk" in name else name[:70]
        d = (e - s) / 1e3
        k = 2 if e > s and covered(s, e) > 0.5 * (e - s) else 0
        acc[key][k] += 1
        acc[key][k + 1] += d
    print("\nkernel, calls alone, mean us alone, calls beside the update, mean us beside, stretch")
    for key, (na, ta, no, to) in sorted(acc.items(), key=lambda x: -(x[1][1] + x[1][3]))[:a.top]:
        ma = ta / na if na else float("nan")
        mo = to / no if no else float("nan")
        print(f"{key}, {na}, {ma:.1f}, {no}, {mo:.1f}, {mo / ma if na and no else float('nan'):.2f}")


if __name__ == "__main__":
    main()
