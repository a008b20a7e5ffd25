"""Per-step breakdown of a rocprofv3 kernel trace of bench.py (steps start at fbank_kernel).

usage: python scripts/analyze_trace.py gpurun_out/prof/run_kernel_trace.csv [--step -2] [--list]
Prints: step wall time, busy time per stream, per-kernel totals for that step, and with --list every
dispatch in order (stream, start offset, duration, grid) — used to find stray copies / gaps.
"""
import argparse
import csv
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    return name.split("(")[0][:90] if not name.startswith("void ") else name[5:].split("(")[0][:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--per-queue", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "fbank_kernel" in r["Kernel_Name"]] + [len(rows)]
    s = a.step
    lo, hi = starts[s - 1], starts[s]
    step = rows[lo:hi]
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    print(f"step {s}: {len(step)} dispatches, wall {(t1 - t0) / 1e3:.1f} us")
    busy = defaultdict(float)
    agg = defaultdict(lambda: [0, 0.0])
    for r in step:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        busy[r["Queue_Id"]] += d
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += d
    for q, b in busy.items():
        print(f"  queue {q}: busy {b:.1f} us")
    # union of busy intervals (any stream)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in step)
    cov, cs, ce = 0, iv[0][0], iv[0][1]
    for a0, a1 in iv[1:]:
        if a0 > ce:
            cov += ce - cs
            cs, ce = a0, a1
        else:
            ce = max(ce, a1)
    cov += ce - cs
    print(f"  GPU busy (union) {cov / 1e3:.1f} us, idle {(t1 - t0 - cov) / 1e3:.1f} us")
    for k, (n, d) in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {d:9.1f} us {n:5d}x {d / n:8.1f} us  {k}")
    if a.per_queue:
        for q in busy:
            qa = defaultdict(lambda: [0, 0.0])
            for r in step:
                if r["Queue_Id"] != q:
                    continue
                d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                qa[short(r["Kernel_Name"])][0] += 1
                qa[short(r["Kernel_Name"])][1] += d
            print(f"== queue {q}")
            for k, (n, d) in sorted(qa.items(), key=lambda x: -x[1][1])[:25]:
                print(f"  {d:9.1f} us {n:5d}x {d / n:8.1f} us  {k}")
    if a.list:
        for r in step:
            st = (int(r["Start_Timestamp"]) - t0) / 1e3
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print(f"q{r['Queue_Id']} {st:9.1f} {d:8.1f}  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}"
                  f" wg {r['Workgroup_Size_X']} vgpr {r['VGPR_Count']}/{r['Accum_VGPR_Count']} "
                  f"lds {r['LDS_Block_Size']}  {short(r['Kernel_Name'])}")


if __name__ == "__main__":
    main()
