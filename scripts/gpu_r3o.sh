#!/bin/bash
# Fused attention backward: unconditional next-head prefetch, scalar key lengths, V fragments
# re-defined after the head-top wait (no compiler vmcnt drains of the register prefetch).
# Bit-identity vs the previous attention build, attention tests, isolated timings, step A/B.
export TMPDIR=/tmp
O=gpurun_out/r3o; mkdir -p $O
L0=multimodal-s2ut_amd/lib/libmms2ut_hip_attnold.so
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 12 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step dump_new 120 python scripts/attn_bits.py /tmp/new.npz
step dump_old 120 env MMS2UT_LIB=$L0 python scripts/attn_bits.py /tmp/old.npz
step cmp 60 python scripts/wgrad_bits.py cmp /tmp/new.npz /tmp/old.npz
step ktests 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread
step attn_new 200 python scripts/attn_bench.py
step attn_old 200 env MMS2UT_LIB=$L0 python scripts/attn_bench.py
step ab 600 python scripts/lib_ab.py $O/attn_ab.json 2 new= attnold=$L0
L2=multimodal-s2ut_amd/lib/libmms2ut_hip_dar.so
step gemm_new 180 python scripts/gemm_bits.py /tmp/g_new.npz
step gemm_dar 180 env MMS2UT_LIB=$L2 python scripts/gemm_bits.py /tmp/g_dar.npz
step gcmp 60 python scripts/wgrad_bits.py cmp /tmp/g_new.npz /tmp/g_dar.npz
step ab2 600 python scripts/lib_ab.py $O/dar_ab.json 2 new= dar=$L2
