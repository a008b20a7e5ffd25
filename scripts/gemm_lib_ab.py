"""Isolated GEMM timings of the step's shapes for alternative library builds (scripts/build_ab.sh).
usage: python scripts/gemm_lib_ab.py name=path [name=path ...]   (path '' = default lib)
Each library runs in its own process (MMS2UT_LIB), twice in mirrored order; per shape the faster of
the two means of 50 warm launches (HIP events), random fp16 operands, the epilogue the step uses for
that projection."""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CHILD = r'''
import importlib, json, sys, torch
sys.path.insert(0, %r)
K = importlib.import_module("multimodal-s2ut_amd").kernels
res = {}
shapes = [("qkv fwd", 10000, 2304, 768, "f16"), ("out-proj fwd", 10000, 768, 768, "drop_resid"),
          ("fc1 fwd", 10000, 3072, 768, "relu_drop"), ("fc2 fwd", 10000, 768, 3072, "drop_resid"),
          ("qkv dgrad", 10000, 768, 2304, "f16"), ("fc1 dgrad", 10000, 768, 3072, "f16"),
          ("fc2 dgrad", 10000, 3072, 768, "relu_drop_bwd"), ("out-proj M11000", 11000, 768, 768, "f16"),
          ("out-proj M12000", 12000, 768, 768, "drop_resid"), ("fc2 fwd M12000", 12000, 768, 3072, "drop_resid"),
          ("qkv dgrad M12000", 12000, 768, 2304, "f16"),
          ("dec fc1 fwd", 3000, 3072, 768, "relu_drop")]
EPI = {"f16": K.EPI_F16, "drop_resid": K.EPI_DROP_RESID, "relu_drop": K.EPI_RELU_DROP, "relu_drop_bwd": K.EPI_RELU_DROP_BWD}
for name, M, N, Kd, epi in shapes:
    A = torch.randn(M, Kd, device="cuda").half(); B = torch.randn(N, Kd, device="cuda").half()
    C = torch.empty(M, N, dtype=torch.float16, device="cuda")
    aux = torch.randn(M, N, device="cuda").half() if epi in ("drop_resid", "relu_drop_bwd") else None
    kw = dict(a_kc=True, b_kc=True, lda=Kd, ldb=Kd, ldc=N, epi=EPI[epi])
    if aux is not None:
        kw.update(aux=aux, ldaux=N)
    if epi != "f16":
        kw.update(p=0.1, seed=5, offset=0, ld_rng=N)
    f = lambda: K.gemm(A, B, C, M, N, Kd, **kw)
    for _ in range(5): f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(50): f()
    e1.record(); torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    res[name] = [round(us, 2), round(2.0 * M * N * Kd / us / 1e6, 1)]
print(json.dumps(res))
'''
# libraries run in A B ... then ... B A order and the faster run per shape is kept: one process per
# library per pass, and the GPU's clock drifts between processes (a later process ran untouched
# shapes 2-6 us slower, profiles/round6_epi_prio_ab.txt)
libs = [a.split("=", 1) for a in sys.argv[1:]]
out = {}
for order in (libs, libs[::-1]):
    for name, path in order:
        env = dict(os.environ)
        if path:
            env["MMS2UT_LIB"] = os.path.join(ROOT, path)
        p = subprocess.run([sys.executable, "-c", CHILD % ROOT], env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if p.returncode or not line:
            print(p.stdout[-2000:], p.stderr[-3000:])
            raise SystemExit(f"{name}: failed rc={p.returncode}")
        res = json.loads(line[-1])
        prev = out.setdefault(name, res)
        for k, v in res.items():
            if v[0] < prev[k][0]:
                prev[k] = v
names = list(out)
print(f"{'shape':18s}" + "".join(f"{n:>22s}" for n in names))
for shape in out[names[0]]:
    print(f"{shape:18s}" + "".join(f"{out[n][shape][0]:10.1f} us {out[n][shape][1]:6.0f} TF" for n in names))
print(json.dumps(out))
