#!/bin/bash
# fbank/CMVN rework check + step trace + bench + SQ PMC passes on three GEMM shapes.
export TMPDIR=/tmp
O=gpurun_out/r3b; mkdir -p $O
step() { local name=$1 secs=$2; shift 2; echo "=== [$name]"; timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1; local rc=$?
         echo "=== [$name] rc=$rc"; tail -n 4 "$O/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step tests 300 python -u -m pytest tests/test_gpu_frontend.py tests/test_gpu_manifest.py -x -q --timeout 120 --timeout-method thread
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-gemm-timing
step bench 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-gemm-timing
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
for shape in "10000 3072 768 1 1" "10000 768 3072 1 1" "10000 768 768 1 1"; do
  tag=$(echo $shape | tr ' ' '_')
  step pmc1_$tag 90 rocprofv3 --pmc $C1 --output-format csv -d $O/pmc1_$tag -o run -- python scripts/gemm_one.py $shape
  step pmc2_$tag 90 rocprofv3 --pmc $C2 --output-format csv -d $O/pmc2_$tag -o run -- python scripts/gemm_one.py $shape
done
