#!/bin/bash
# Repeated A/B of the LayerNorm-backward rows per block (MMS2UT_LN_NP = 1 vs 2), training step only.
mkdir -p gpurun_out
for r in 1 2 3; do
for np in 2 1; do
  MMS2UT_LN_NP=$np timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-gemm-timing > gpurun_out/lnab_$np.log 2>&1 || exit 1
  echo "NP=$np $(tail -1 gpurun_out/lnab_$np.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
