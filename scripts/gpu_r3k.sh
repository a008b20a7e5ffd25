#!/bin/bash
# Weight-gradient k-loop: fragment reads before the next stage's DMA (no compiler vmcnt(0) in front
# of the transpose reads): bit-identity vs the previous build (wg0), isolated wgrad timings, kernel
# tests, step A/B.
export TMPDIR=/tmp
O=gpurun_out/r3k; mkdir -p $O
W0=multimodal-s2ut_amd/lib/libmms2ut_hip_wg0.so
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 8 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step dump_new 120 python scripts/wgrad_bits.py dump /tmp/new.npz
step dump_old 120 env MMS2UT_LIB=$W0 python scripts/wgrad_bits.py dump /tmp/old.npz
step cmp 60 python scripts/wgrad_bits.py cmp /tmp/new.npz /tmp/old.npz
step ktests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_splitk.py -x -q --timeout 120 --timeout-method thread
step wg_new 120 python scripts/wgrad_ab.py
step wg_old 120 env MMS2UT_LIB=$W0 python scripts/wgrad_ab.py
step ab 600 python scripts/lib_ab.py $O/wg_ab.json 2 rf= wg0=$W0
