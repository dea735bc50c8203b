#!/usr/bin/env python
"""Summarise rocprofv3 --pmc CSV output per kernel: counters summed over dispatches, plus the ratios
used in profiles/attn_pmc_*.txt (SQ_* time counters are quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES and
GRBM_GUI_ACTIVE cycles; MI355X_MICROARCH.md 'DVFS give-back').

  python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 [--filter attn]
"""
import argparse
import collections
import csv
import glob
import os


def load(dirs, filt):
    sums = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = row.get("Kernel_Name", "?")
                    if filt and filt not in k:
                        continue
                    sums[k][row["Counter_Name"]] += float(row["Counter_Value"])
                    disp[k].add((f, row.get("Dispatch_Id")))
                    meta[k] = (row.get("VGPR_Count") or row.get("Arch_VGPR_Count"), row.get("Accum_VGPR_Count"),
                               row.get("LDS_Block_Size"))
    return sums, disp, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    sums, disp, meta = load(a.dirs, a.filter)
    for k in sorted(sums, key=lambda x: -sums[x].get("SQ_WAVE_CYCLES", 0)):
        c = sums[k]
        v, ag, lds = meta[k]
        print(f"{k[:110]}  (VGPR {v}, AGPR {ag}, LDS {lds} B, {len(disp[k])} dispatch-passes)")
        for n in sorted(c):
            print(f"  {n:28s} {c[n]:.4g}")
        w = c.get("SQ_WAVE_CYCLES")
        if w:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
                if n in c:
                    print(f"  {n} / wave cycles = {c[n] / w:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in c and "SQ_LDS_IDX_ACTIVE" in c and c["SQ_LDS_IDX_ACTIVE"]:
            print(f"  LDS bank-conflict cycles / LDS-array cycles = {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c and c["GRBM_GUI_ACTIVE"]:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; MFMA busy sums the 1024 SIMDs
            print(f"  MFMA busy per SIMD / GPU-active cycles = "
                  f"{(c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024) / (c['GRBM_GUI_ACTIVE'] / 8):.3f}")
        print()


if __name__ == "__main__":
    main()
