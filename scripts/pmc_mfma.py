"""MFMA utilisation of the training step's kernels from one rocprofv3 PMC pass over bench.py
(counters SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES — one pass, within the SQ /
GRBM slot limits of MI355X_MICROARCH.md).  Windows are fbank launch to fbank launch (one training
step each); bench.py cycles through its resident batches (a K=3 window holds 3 batches, one of
them the dataset's short tail batch), so the figures aggregate the last complete cycle of
--cycle windows (default 3), and each window is reported on its own.

  MFMA utilisation of a kernel = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs × 256 CUs × 4 SIMDs)

i.e. the fraction of all SIMD-cycles of the kernel's duration in which the matrix pipe was busy
(dense-peak-relative: 16x16x32 f16 MFMA = 16 cycles per SIMD at 2.5 PF/s chip-wide).  PMC passes
serialise kernels, so the side-stream overlap of the real step is absent here.

usage: python scripts/pmc_mfma.py PMC_DIR [--out profiles/roundN_mfma_util.json]
"""
import argparse
import csv
import json
import re
from collections import defaultdict


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", n)
    return n.split("(")[0][:80] if not n.startswith("void ") else n[5:].split("(")[0][:80]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc")
    ap.add_argument("--out", default=None)
    ap.add_argument("--cycle", type=int, default=3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.pmc + "/run_counter_collection.csv")))
    per = defaultdict(dict)
    names = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    order = sorted(per)
    starts = [d for d in order if "fbank_kernel" in names[d]]
    lo, hi = starts[-1 - a.cycle], starts[-1]
    step = [d for d in order if lo <= d < hi]
    windows = []
    for w0, w1 in zip(starts[-1 - a.cycle:-1], starts[-a.cycle:]):
        ds = [d for d in order if w0 <= d < w1]
        b = sum(per[d].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in ds)
        g = sum(per[d].get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256 * 4 for d in ds)
        gd = [d for d in ds if short(names[d]).startswith("gemm")]
        gb = sum(per[d].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in gd)
        gg = sum(per[d].get("GRBM_GUI_ACTIVE", 0.0) / 8 * 256 * 4 for d in gd)
        windows.append({"dispatches": len(ds), "mfma_util": b / max(g, 1.0), "gemm_mfma_util": gb / max(gg, 1.0),
                        "mfma_busy": b})
        print(f"window {w0}: {len(ds)} dispatches, MFMA util {b / max(g, 1.0) * 100:.1f} % "
              f"(GEMMs {gb / max(gg, 1.0) * 100:.1f} %)")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    tot = [0.0, 0.0]
    for d in step:
        c = per[d]
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0)
        k = short(names[d])
        agg[k][0] += 1
        agg[k][1] += busy
        agg[k][2] += gui / 8 * 256 * 4
        tot[0] += busy
        tot[1] += gui / 8 * 256 * 4
    out = {"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES of "
                     "`python bench.py --steps 3 --warmup 1 --no-gemm-timing`; the last cycle of "
                     f"{a.cycle} training steps (bench's resident batches)",
           "formula": "MFMA_BUSY / (GRBM_GUI_ACTIVE/8 * 256 CU * 4 SIMD)",
           "step_mfma_util": tot[0] / max(tot[1], 1.0), "windows": windows, "per_kernel": {}}
    gemm = [0.0, 0.0]
    for k, (n, b, g) in sorted(agg.items(), key=lambda kv: -kv[1][2]):
        out["per_kernel"][k] = {"launches": n, "mfma_util": b / max(g, 1.0), "simd_cycles": g}
        if k.startswith("gemm"):
            gemm[0] += b
            gemm[1] += g
    out["gemm_mfma_util"] = gemm[0] / max(gemm[1], 1.0)
    for k, v in list(out["per_kernel"].items())[:16]:
        print(f"{v['mfma_util']*100:6.1f} %  {v['launches']:4d}x  {k}")
    print(f"all GEMM launches: {out['gemm_mfma_util']*100:.1f} %   whole step: {out['step_mfma_util']*100:.1f} %")
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
