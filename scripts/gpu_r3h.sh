#!/bin/bash
# token-embedding scatter rewrite + transpose descriptor search: tests, step A/B vs the previous build, kernel stats
export TMPDIR=/tmp
O=gpurun_out/r3h; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 6 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_layers.py
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-gemm-timing
step step 600 python scripts/lib_ab.py $O/step_ab.json 2 new= old=multimodal-s2ut_amd/lib/libmms2ut_hip_old.so
