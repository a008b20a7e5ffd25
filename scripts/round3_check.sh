#!/bin/bash
# GPU check of HEAD: GPU tests, smoke, default bench line, rocprofv3 kernel trace + stats of the
# bench. Each step under its own limit; stop at the first crash / timeout.  Outputs in $1.
export TMPDIR=/tmp
O=${1:-gpurun_out/r3}
mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 6 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step tests 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 240 python bench.py
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
