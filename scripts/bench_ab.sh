#!/bin/bash
# Run bench.py under several environment settings in one GPU call; one summary line per variant.
# usage: scripts/bench_ab.sh "NAME:ENV=V ENV2=V" ...   (each variant its own 240-s limit)
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  env $envs timeout -k 10 240 python bench.py --no-cpu-baseline --steps 12 --warmup 3 > "gpurun_out/ab_$name.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc"; tail -5 "gpurun_out/ab_$name.log"; exit $rc; fi
  python - "$name" "gpurun_out/ab_$name.log" << 'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
r = d["roofline"]
print(f"[{sys.argv[1]:14s}] {d['ms_per_step']:7.2f} ms/step  {d['value']/1e6:6.3f} Mframes/s  gemm {r['gemm_ms_per_step']:6.2f} ms  ach {r['achieved']:6.1f} TF  issue {r['host_issue_ms_per_step']:5.2f} ms  host cpu {r.get('host_cpu_ms_per_step', float('nan')):5.2f} ms", flush=True)
PY
done
