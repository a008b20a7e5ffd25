#!/bin/bash
# One GPU call that produces the round's evidence: PMC HBM traffic (two separate passes), a kernel
# trace with per-kernel stats, and the default bench line.  Outputs under gpurun_out/round/.
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gemm-timing"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B > $O/pmc_fetch.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B > $O/pmc_write.log 2>&1 || { echo "write pass failed"; tail -5 $O/pmc_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "trace failed"; tail -5 $O/trace.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
