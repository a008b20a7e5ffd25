#!/bin/bash
# SQ / TCC counters of the fused attention kernels on one shape (scripts/attn_bench.py B T p causal).
# usage: scripts/_pmc_attn.sh "B T p causal" TAG
export TMPDIR=/tmp
shape="$1"; tag="$2"
C1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
C2="SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE GRBM_COUNT"
C3="FETCH_SIZE"
C4="WRITE_SIZE"
for i in 1 2 3 4; do
  eval C=\$C$i
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${tag}_$i -o run -- python scripts/attn_bench.py $shape > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pmc $tag $i failed"; tail -3 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
echo done
