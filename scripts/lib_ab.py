"""Step-time A/B of alternative library builds (scripts/build_ab.sh): one bench.py run per library,
interleaved `reps` times, plus the isolated LayerNorm-backward timings of ops_bench for each.
usage: python scripts/lib_ab.py OUT_JSON REPS name=path [name=path ...]   (path '' = default lib)"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
out, reps = sys.argv[1], int(sys.argv[2])
libs = [a.split("=", 1) for a in sys.argv[3:]]
res = {}
for rep in range(reps):
    for name, path in libs:
        env = dict(os.environ)
        if path:
            env["MMS2UT_LIB"] = os.path.join(ROOT, path)
        if rep == 0:
            p = subprocess.run([sys.executable, os.path.join(HERE, "ops_bench.py")], env=env, capture_output=True,
                               text=True, timeout=200)
            ln = [l for l in p.stdout.splitlines() if l.startswith("layernorm")]
            res.setdefault(name, {})["ops"] = ln
            print(name, *ln, sep="\n  ", flush=True)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
                            "--no-cpu-baseline", "--no-gemm-timing"], env=env, capture_output=True, text=True,
                           timeout=300, cwd=ROOT)
        line = [l for l in p.stdout.splitlines() if l.startswith("{")]
        if p.returncode or not line:
            print(p.stdout[-2000:], p.stderr[-2000:])
            raise SystemExit(f"{name}: bench failed rc={p.returncode}")
        d = json.loads(line[-1])
        ms, ck = d["ms_per_step"], d.get("optimizer", {}).get("master_checksum")
        res.setdefault(name, {}).setdefault("ms", []).append(ms)
        res[name].setdefault("master_checksum", []).append(ck)
        print(f"{name:12s} rep {rep}: {ms:.3f} ms/step  master checksum {ck!r}", flush=True)
json.dump(res, open(out, "w"), indent=1)
