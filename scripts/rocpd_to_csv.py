"""Convert a rocprofv3 rocpd database (ROCm 7.2's default output, run_results.db) into the
kernel-trace CSV layout the trace scripts read (analyze_trace.py, trace_gaps.py, trace_totals.py).
usage: python scripts/rocpd_to_csv.py DIR/run_results.db [OUT.csv]   (default: DIR/run_kernel_trace.csv)"""
import csv
import os
import sqlite3
import sys

db = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(db), "run_kernel_trace.csv")
c = sqlite3.connect(db)
rows = c.execute("select name, start, end, queue_id, stream_id, grid_x, grid_y, grid_z, workgroup_x, dispatch_id "
                 "from kernels order by start").fetchall()
with open(out, "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id", "Stream_Id", "Grid_Size",
                "Workgroup_Size", "Dispatch_Id"])
    for n, s, e, q, st, gx, gy, gz, wx, d in rows:
        w.writerow([n, s, e, q, st, gx * gy * gz, wx, d])
print(f"{len(rows)} dispatches -> {out}")
