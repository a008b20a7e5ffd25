#!/bin/bash
# Repeated A/B of the weight-gradient split-K block budget (MMS2UT_WGRAD_SLOTS) in the training step.
mkdir -p gpurun_out
for r in 1 2 3; do
for v in 512 256 1024; do
  MMS2UT_WGRAD_SLOTS=$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-gemm-timing > gpurun_out/wsab.log 2>&1 || exit 1
  echo "SLOTS=$v $(tail -1 gpurun_out/wsab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
