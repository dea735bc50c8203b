#!/usr/bin/env python
"""Effective clock per kernel from a rocprofv3 GRBM PMC run (rocpd SQLite output):
GRBM_GUI_ACTIVE / 8 XCDs / kernel duration, median over dispatches longer than 0.3 ms (shorter
ones read high, MI355X_MICROARCH.md 'DVFS give-back').

  rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc_clock -o run -- python3 bench.py ...
  python tools/pmc_clock.py gpurun_out/pmc_clock/run_results.db
"""
import collections
import sqlite3
import statistics
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    d = collections.defaultdict(dict)
    q = "select dispatch_id, kernel_name, grid_size, counter_name, value, duration from counters_collection"
    for disp, name, grid, cn, val, dur in c.execute(q):
        d[disp].update(name=name, grid=grid, dur=dur)
        d[disp][cn] = val
    g = collections.defaultdict(list)
    for v in d.values():
        if v["dur"] < 300000 or "GRBM_GUI_ACTIVE" not in v:
            continue
        n = "GEMM(lib) grid %d" % v["grid"] if "Cijk" in v["name"] else v["name"][:50]
        g[n].append((v["GRBM_GUI_ACTIVE"] / 8 / v["dur"], v["dur"] / 1e6))
    print("kernel, dispatches, median effective clock GHz, median ms")
    for n, vals in sorted(g.items(), key=lambda x: -sum(t[1] for t in x[1])):
        print("%-55s %4d  %.2f  %.3f" % (n, len(vals), statistics.median(t[0] for t in vals),
                                         statistics.median(t[1] for t in vals)))


if __name__ == "__main__":
    main()
