"""Idle time of a rocprofv3 kernel trace of bench.py: per optimizer step, the wall time, the summed
kernel time, the time some kernel is running on any queue (busy), and the largest idle gaps with
the kernels on either side.  usage: python scripts/trace_gaps.py run_kernel_trace.csv [N] [SKIP] [TOP]
(N steps ending SKIP steps before the last fbank launch; bench.py's serial roofline pass follows
its timed pass, so SKIP = N selects the timed pass)."""
import csv
import re
import sys
from collections import Counter

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
top = int(sys.argv[4]) if len(sys.argv) > 4 else 12
starts = [i for i, r in enumerate(rows) if "fbank_kernel" in r["Kernel_Name"]]
seg = rows[starts[-n - 1 - skip]: starts[-1 - skip]]


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    return (name[5:] if name.startswith("void ") else name).split("(")[0][:48]


t0, t1 = int(seg[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in seg)
tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
busy, gaps = 0, []
cs, ce, last = int(seg[0]["Start_Timestamp"]), int(seg[0]["End_Timestamp"]), seg[0]
for r in seg[1:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s > ce:
        busy += ce - cs
        gaps.append(((s - ce) / 1e3, short(last["Kernel_Name"]), short(r["Kernel_Name"])))
        cs, ce, last = s, e, r
    elif e > ce:
        ce, last = e, r
busy += ce - cs
print(f"{n} steps: wall {(t1 - t0) / 1e3 / n:.1f} us/step, summed kernels {tot / 1e3 / n:.1f}, busy {busy / 1e3 / n:.1f}, "
      f"idle {(t1 - t0 - busy) / 1e3 / n:.1f} us/step in {len(gaps) / n:.1f} gaps")
pairs = Counter()
for g, a, b in gaps:
    pairs[(a, b)] += g
print("idle us/step by (kernel before, kernel after):")
for (a, b), g in pairs.most_common(top):
    print(f"  {g / n:8.1f}  {a:48s} -> {b}")
