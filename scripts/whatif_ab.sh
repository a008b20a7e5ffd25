#!/bin/bash
# bench.py variants with dropout rates forced to 0 (scripts/whatif_dropout.py), one summary line each
# usage: scripts/whatif_ab.sh "NAME:key1,key2" ...   (empty key list = unchanged)
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; keys="${spec#*:}"
  WHATIF="$keys" timeout -k 10 240 python scripts/whatif_dropout.py --no-cpu-baseline --steps 12 --warmup 3 --no-gemm-timing > "gpurun_out/wi_$name.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc"; tail -5 "gpurun_out/wi_$name.log"; exit $rc; fi
  python - "$name" "gpurun_out/wi_$name.log" << 'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(f"[{sys.argv[1]:10s}] {d['ms_per_step']:7.2f} ms/step", flush=True)
PY
done
