export TMPDIR=/tmp
MMS2UT_GEMM_BK=32 timeout -k 10 200 python -m pytest tests/test_gpu_kernels.py -q -x -k gemm > gpurun_out/kt32.log 2>&1; echo "kt32 rc=$?"; tail -2 gpurun_out/kt32.log
timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gb.log 2>&1; echo "gb rc=$?"
