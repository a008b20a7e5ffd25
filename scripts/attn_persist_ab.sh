#!/bin/bash
# Repeated A/B of the fused attention backward grid in the training step: persistent (one block per
# CU, default) vs one block per head (MMS2UT_ATTN_PERSIST=0).
mkdir -p gpurun_out
for r in 1 2 3; do
for v in default 0; do
  if [ "$v" = default ]; then unset MMS2UT_ATTN_PERSIST; else export MMS2UT_ATTN_PERSIST=$v; fi
  timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-gemm-timing > gpurun_out/apab.log 2>&1 || exit 1
  echo "PERSIST=$v $(tail -1 gpurun_out/apab.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
