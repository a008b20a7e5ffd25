"""HBM traffic of the GEMM launches from two rocprofv3 PMC passes of bench.py (FETCH_SIZE, WRITE_SIZE;
separate passes as MI355X_MICROARCH.md §HBM / §PMC slots prescribe; FETCH_SIZE doubled for gfx950's
half-counted 128-B requests).  Mean over the complete steps after the first.

usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR [--out profiles/roundN_gemm_traffic.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def load(path):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return rows


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    return n.replace("void ", "").split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    F = load(a.fetch + "/run_counter_collection.csv")
    W = {r["Dispatch_Id"]: float(r["Counter_Value"]) for r in load(a.write + "/run_counter_collection.csv")}
    # steps start at the fbank launch (the optimizer is chunked and deferred into the next step);
    # every complete step after the first (warm-up) one is averaged, so batches of every length
    # bucket count in proportion
    starts = [i for i, r in enumerate(F) if "fbank_kernel" in r["Kernel_Name"]]
    first = 1 if len(starts) > 2 else 0
    nsteps = len(starts) - 1 - first
    step = F[starts[first]: starts[-1]]
    per = defaultdict(lambda: [0, 0.0, 0.0])
    tot = [0.0, 0.0]
    for r in step:
        k = short(r["Kernel_Name"])
        fetch = 2.0 * float(r["Counter_Value"]) * 1024  # gfx950: FETCH_SIZE counts 128-B requests as 64 B
        write = W.get(r["Dispatch_Id"], 0.0) * 1024
        per[k][0] += 1
        per[k][1] += fetch
        per[k][2] += write
        tot[0] += fetch
        tot[1] += write
    # a GEMM call is its gemm launch plus, for split-K forward / dgrad GEMMs, its fixup pass
    gemm = [(k, v) for k, v in per.items() if "gemm" in k or "splitk_fixup" in k]
    gl = sum(v[0] for k, v in gemm if "gemm" in k) / nsteps
    gb = sum(v[1] + v[2] for _, v in gemm) / nsteps
    for v in per.values():
        v[0] /= nsteps
        v[1] /= nsteps
        v[2] /= nsteps
    tot = [t / nsteps for t in tot]
    out = {
        "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
                  "`python bench.py --steps 3 --warmup 1`; mean over the complete steps after the first; "
                  "FETCH x2 (gfx950); GEMM = gemm launches + their split-K fixup passes",
        "steps_averaged": nsteps,
        "step_dispatches": len(step) / nsteps,
        "step_hbm_bytes": tot[0] + tot[1],
        "gemm_launches": gl,
        "gemm_hbm_bytes_per_step": gb,
        "gemm_hbm_bytes_per_launch": gb / max(gl, 1),
        "per_kernel": {k: {"launches": v[0], "read_bytes": v[1], "write_bytes": v[2],
                           "bytes_per_launch": (v[1] + v[2]) / v[0]}
                       for k, v in sorted(per.items(), key=lambda x: -(x[1][1] + x[1][2]))},
    }
    print(json.dumps({k: v for k, v in out.items() if k != "per_kernel"}, indent=1))
    for k, v in list(out["per_kernel"].items())[:20]:
        print(f"{v['read_bytes'] / 1e6:9.1f} MB rd {v['write_bytes'] / 1e6:9.1f} MB wr {v['launches']:6.1f}x  {k}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
