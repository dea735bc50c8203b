"""Export the kernel dispatches of a rocprofv3 SQLite output (``rocprofv3 -d DIR -o run`` writes
DIR/run_results.db) to the kernel-trace CSV columns tools/trace_summary.py reads.

    python tools/rocpd_to_csv.py gpurun_out/prof/run_results.db out.csv
"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, queue_id, grid_x, grid_y, grid_z, workgroup_x, lds_size, "
                     "vgpr_count, accum_vgpr_count from kernels order by start").fetchall()
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Grid_Size_X", "Grid_Size_Y",
                    "Grid_Size_Z", "Workgroup_Size_X", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count"])
        w.writerows(rows)
    print(f"{len(rows)} dispatches -> {out}")


if __name__ == "__main__":
    main()
