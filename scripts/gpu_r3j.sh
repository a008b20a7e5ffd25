#!/bin/bash
# LayerNorm-backward one-wave-per-row kernel: GPU tests with it, isolated LN timings + step A/B vs
# the half-wave kernel (ln0) and the two-rows-per-iteration form (ln2); smoke; kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r3j; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 5 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step ab 900 python scripts/lib_ab.py $O/ln_ab.json 2 w1= ln0=multimodal-s2ut_amd/lib/libmms2ut_hip_ln0.so ln2=multimodal-s2ut_amd/lib/libmms2ut_hip_ln2.so
step bench 300 python bench.py
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline
