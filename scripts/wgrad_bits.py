"""Dump the grouped weight-gradient outputs of one seeded encoder-layer problem set (library under
test: MMS2UT_LIB) to an .npz, or compare two such dumps bit for bit.
usage: python scripts/wgrad_bits.py dump OUT.npz [rows] | python scripts/wgrad_bits.py cmp A.npz B.npz"""
import importlib
import os
import sys

import numpy as np

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k].view(np.uint16), b[k].view(np.uint16))]
    print("bit-identical" if not bad else f"DIFFER: {bad}", f"({len(a.files)} arrays)")
    sys.exit(1 if bad else 0)
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
K = importlib.import_module("multimodal-s2ut_amd").kernels
out = {}
for rows in ([int(sys.argv[3])] if len(sys.argv) > 3 else [10000, 777, 31]):
    g = torch.Generator(device="cuda").manual_seed(rows)
    probs = []
    for N, Kin, bias in [(2304, 768, True), (768, 768, True), (3072, 768, True), (768, 3072, True), (200, 136, False)]:
        dy = (torch.randn(rows, N, device="cuda", generator=g) * 0.1).half()
        x = torch.randn(rows, Kin, device="cuda", generator=g).half()
        dW = torch.empty(N, Kin, dtype=torch.float16, device="cuda")
        db = torch.empty(N, dtype=torch.float16, device="cuda") if bias else None
        probs.append((dy, x, dW, db))
    K.wgrad_group(probs, rows)
    torch.cuda.synchronize()
    for i, (_, _, dW, db) in enumerate(probs):
        out[f"r{rows}_p{i}_dW"] = dW.cpu().numpy()
        if db is not None:
            out[f"r{rows}_p{i}_db"] = db.cpu().numpy()
np.savez(sys.argv[2], **out)
print("dumped", len(out), "arrays to", sys.argv[2])
