#!/bin/bash
# GEMM time by shape class in the step (roofline pass dump) + isolated epilogue costs at M = 10000.
export TMPDIR=/tmp
O=gpurun_out/r3d; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step dump 300 env MMS2UT_GEMM_DUMP=$O/gemm.npz python bench.py --steps 5 --warmup 2 --no-cpu-baseline
step table 60 python scripts/gemm_table.py $O/gemm.npz
step epi 200 python scripts/gemm_epi.py 10000
