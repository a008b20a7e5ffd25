#!/bin/bash
# Round-3 evidence in one GPU call: GPU tests + smoke, default bench line, two PMC passes
# (FETCH_SIZE / WRITE_SIZE) for the GEMM HBM traffic, the gloo DP2 rehearsal of the N>1 bench path,
# a rocprofv3 kernel trace + stats of the bench, and attention timings with / without dropout.
# Each step under its own limit; stop at the first crash / timeout.  Outputs under $1.
export TMPDIR=/tmp
O=${1:-gpurun_out/ev6}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step tests 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-gemm-timing"
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python $B
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python $B
step traffic 60 python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write --out $O/gemm_traffic.json

step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline



step dp2 600 scripts/_dp2_rehearsal.sh $O/dp2
