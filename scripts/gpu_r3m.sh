#!/bin/bash
# NT GEMM 32-deep 5-slot ring (ra0 build) vs the BK=64 2-stage tile: bit-identity, isolated
# times on the step's shapes, step A/B.
export TMPDIR=/tmp
O=gpurun_out/r3m; mkdir -p $O
L1=multimodal-s2ut_amd/lib/libmms2ut_hip_ra0.so
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 8 "$O/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step base 180 python scripts/gemm_bits.py /tmp/base.npz
step ring 180 env MMS2UT_LIB=$L1 python scripts/gemm_bits.py /tmp/ring.npz
step cmp 60 python scripts/wgrad_bits.py cmp /tmp/base.npz /tmp/ring.npz
step ab 600 python scripts/lib_ab.py $O/ring_ab.json 2 base= ra0=$L1
