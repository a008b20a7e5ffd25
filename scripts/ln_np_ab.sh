#!/bin/bash
# A/B of the LayerNorm-backward rows per block (MMS2UT_LN_NP = row pairs per wave: 8*NP rows per block):
# LN parity tests, isolated kernel timings and the training step for each setting.
mkdir -p gpurun_out
for np in 2 1 4; do
  export MMS2UT_LN_NP=$np
  echo "=== NP=$np"
  timeout -k 10 120 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q -k "layernorm or model" --timeout 100 --timeout-method thread > gpurun_out/ln_np$np.test.log 2>&1 || { echo "tests failed NP=$np"; tail -20 gpurun_out/ln_np$np.test.log; exit 1; }
  tail -1 gpurun_out/ln_np$np.test.log
  timeout -k 10 120 python scripts/ops_bench.py 2>/dev/null | grep layernorm_bwd || exit 1
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-gemm-timing --steps 20 > gpurun_out/ln_np$np.bench.log 2>&1 || exit 1
  tail -1 gpurun_out/ln_np$np.bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', round(d['ms_per_step'],3), 'value', round(d['value']))"
done
