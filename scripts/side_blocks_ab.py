"""A/B of the grid cap of the grouped weight-gradient launches on the side stream
(kernels.SIDE_WGRAD_BLOCKS): one bench.py run per value, interleaved twice.  cap -1: no side stream
(every side job in order on the main stream).
usage: python scripts/side_blocks_ab.py OUT_JSON [caps...]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
out = sys.argv[1]
caps = [int(c) for c in sys.argv[2:]] or [0, 128, 64, 256]
child = ("import sys, runpy; sys.path.insert(0, {root!r}); import importlib; "
         "K = importlib.import_module('multimodal-s2ut_amd').kernels; K.SIDE_WGRAD_BLOCKS = max({cap}, 0); K._Side.enabled = {cap} >= 0; "
         "sys.argv = ['bench.py', '--steps', '20', '--warmup', '5', '--no-cpu-baseline', '--no-gemm-timing']; "
         "runpy.run_path({bench!r}, run_name='__main__')")
res = {}
for rep in range(2):
    for cap in caps:
        p = subprocess.run([sys.executable, "-c", child.format(root=ROOT, cap=cap, bench=os.path.join(ROOT, "bench.py"))],
                           capture_output=True, text=True, timeout=300)
        line = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if p.returncode or not line:
            print(p.stdout[-2000:], p.stderr[-2000:])
            raise SystemExit(f"cap {cap}: bench failed rc={p.returncode}")
        ms = json.loads(line[-1])["ms_per_step"]
        res.setdefault(cap, []).append(ms)
        print(f"cap {cap:4d} rep {rep}: {ms:.3f} ms/step", flush=True)
json.dump(res, open(out, "w"), indent=1)
