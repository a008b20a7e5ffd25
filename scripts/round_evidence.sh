#!/bin/bash
# Round-end evidence in one GPU call: GPU tests + smoke, bench line, rocprofv3 kernel trace/stats of
# the default bench, two PMC passes (FETCH_SIZE / WRITE_SIZE) for the GEMM HBM traffic.  Outputs
# under gpurun_out/ev/; each step under its own time limit, stop at the first crash / timeout.
export TMPDIR=/tmp
O=gpurun_out/ev
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python bench.py
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gemm-timing"
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B
step dp2 300 scripts/_dp2_rehearsal.sh
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
