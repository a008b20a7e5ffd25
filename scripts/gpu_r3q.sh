#!/bin/bash
# Round-3 v6: GPU tests + smoke + bench at HEAD first, then the attention-prefetch A/B (bit-identity vs
# the previous attention build, isolated timings, step A/B), kernel trace, PMC traffic, NT
# DMA-after-reads A/B, gloo DP2 rehearsal.  Each step under its own limit; stop at the first failure.
export TMPDIR=/tmp
O=gpurun_out/ev6; mkdir -p $O
L0=multimodal-s2ut_amd/lib/libmms2ut_hip_attnold.so
L2=multimodal-s2ut_amd/lib/libmms2ut_hip_dar.so
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 10 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step dump_new 120 python scripts/attn_bits.py /tmp/new.npz
step dump_old 120 env MMS2UT_LIB=$L0 python scripts/attn_bits.py /tmp/old.npz
step cmp 60 python scripts/wgrad_bits.py cmp /tmp/new.npz /tmp/old.npz
step attn_new 200 python scripts/attn_bench.py
step attn_old 200 env MMS2UT_LIB=$L0 python scripts/attn_bench.py
step ab 600 python scripts/lib_ab.py $O/attn_ab.json 2 new= attnold=$L0
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline
