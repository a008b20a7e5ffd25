"""Mean PMC counter values per (kernel, grid size) from a rocprofv3 --pmc run directory (or its
run_counter_collection.csv).  FETCH_SIZE is reported in bytes, doubled for gfx950's half-counted
128-B requests (MI355X_MICROARCH.md); other counters raw.
usage: python scripts/pmc_dispatch.py DIR [DIR ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    path = d if d.endswith(".csv") else (glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True) or [d])[0]
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).replace("void ", "").split("(")[0][:60]
        key = (k, int(r.get("Grid_Size", 0) or 0))
        v = float(r["Counter_Value"])
        if r["Counter_Name"] == "FETCH_SIZE":
            v *= 2048.0
        elif r["Counter_Name"] == "WRITE_SIZE":
            v *= 1024.0
        acc[key][r["Counter_Name"]].append(v)
    print(f"== {path}")
    for (k, grid), cs in sorted(acc.items(), key=lambda kv: kv[0][1]):
        if "gemm" not in k:
            continue
        parts = [f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())]
        print(f"  {k:60s} grid {grid:8d}  n={len(next(iter(cs.values())))}  " + "  ".join(parts))
