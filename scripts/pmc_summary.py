"""Summarise rocprofv3 --pmc CSVs: per kernel name, mean of each counter over dispatches.
usage: python scripts/pmc_summary.py DIR [DIR...] [--match SUBSTR]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args.remove(match)
for d in args:
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        acc[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {d}")
    for k, cs in acc.items():
        n = max(len(v) for v in cs.values())
        print(f"  {k}  (n={n})")
        for c, v in sorted(cs.items()):
            print(f"     {c:28s} {sum(v) / len(v):16.4g}")
