#!/bin/bash
# fbank rework check (default lib) + the BK=32 high-occupancy GEMM A/B (occ2 / occ3 libraries).
export TMPDIR=/tmp
O=gpurun_out/r3c; mkdir -p $O
L=multimodal-s2ut_amd/lib
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step fe 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_manifest.py -x -q --timeout 120 --timeout-method thread
step gemm_occ2 300 env MMS2UT_LIB=$L/libmms2ut_hip_occ2.so python -u -m pytest tests/test_gpu_gemm_splitk.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or linear or splitk"
step gemm_occ3 300 env MMS2UT_LIB=$L/libmms2ut_hip_occ3.so python -u -m pytest tests/test_gpu_gemm_splitk.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "gemm or linear or splitk"
step gemm_ab 300 python scripts/gemm_lib_ab.py base= occ2=$L/libmms2ut_hip_occ2.so occ3=$L/libmms2ut_hip_occ3.so
step step_ab 600 python scripts/lib_ab.py $O/step_ab.json 2 base= occ2=$L/libmms2ut_hip_occ2.so occ3=$L/libmms2ut_hip_occ3.so
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-gemm-timing
