mkdir -p gpurun_out
timeout -k 10 200 python -m pytest tests/test_gpu_model.py tests/test_gpu_trainer.py -x -q --timeout 100 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -20 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for r in 1 2; do
for v in 1 0; do
  MMS2UT_DGRAD_FIRST=$v timeout -k 10 200 python bench.py --steps 20 --no-cpu-baseline --no-gemm-timing > gpurun_out/ab_$v.log 2>&1 || exit 1
  echo "DGRAD_FIRST=$v $(tail -1 gpurun_out/ab_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3))')"
done
done
