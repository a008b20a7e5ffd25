#!/bin/bash
# Re-entry check at HEAD: all GPU tests + smoke, default bench line, kernel trace + stats of the bench.
export TMPDIR=/tmp
O=gpurun_out/r3i; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline
