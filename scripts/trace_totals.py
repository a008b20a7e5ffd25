"""Per-kernel totals over the last N optimizer steps of a rocprofv3 kernel trace of bench.py, split
by queue (main vs side stream).  usage: python scripts/trace_totals.py run_kernel_trace.csv [N] [SKIP]
SKIP: leave out the last SKIP steps (bench.py's serial roofline pass follows its timed pass)."""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    return name.split("(")[0][:70] if not name.startswith("void ") else name[5:].split("(")[0][:70]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
starts = [i for i, r in enumerate(rows) if "fbank_kernel" in r["Kernel_Name"]]
rows = rows[starts[-n - 1 - skip]: starts[-1 - skip]]
t0, t1 = int(rows[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in rows)
print(f"{n} steps, wall {(t1 - t0) / 1e3 / n:.1f} us/step")
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(lambda: defaultdict(int))
for r in rows:
    k = short(r["Kernel_Name"])
    agg[r["Queue_Id"]][k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / n
    cnt[r["Queue_Id"]][k] += 1
print("   us/step  launches/step  us/launch  kernel")
for q, d in sorted(agg.items(), key=lambda kv: -sum(kv[1].values())):
    print(f"== queue {q}: {sum(d.values()):.1f} us/step")
    for k, v in sorted(d.items(), key=lambda kv: -kv[1])[:25]:
        c = cnt[q][k] / n
        print(f"  {v:9.1f}  {c:9.1f}  {v / c:9.1f}  {k}")
