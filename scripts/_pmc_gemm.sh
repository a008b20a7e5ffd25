export TMPDIR=/tmp
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"
for shape in "10000 3072 768 1 1" "10000 768 3072 1 0" "3072 768 10000 0 0 8"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --pmc $C1 --output-format csv -d gpurun_out/pg1_$tag -o run -- python scripts/gemm_one.py $shape > /dev/null 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc $C2 --output-format csv -d gpurun_out/pg2_$tag -o run -- python scripts/gemm_one.py $shape > /dev/null 2>&1 || exit 1
done
echo done
