#!/bin/bash
# Kernel trace of the overlapped training step only (no roofline pass, no CPU baseline) + isolated
# HBM-bound kernel timings.  Outputs under $1 (default gpurun_out/tr).
export TMPDIR=/tmp
O=${1:-gpurun_out/tr}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
[ -n "$TESTS" ] && step tests 300 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-gemm-timing
step ops 200 python scripts/ops_bench.py
