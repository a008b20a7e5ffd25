set -o pipefail
O=gpurun_out/r4d; L=multimodal-s2ut_amd/lib
scripts/ab_env.sh $O "python scripts/gemm_l2_ab.py" "base:MMS2UT_GEMM_PP=0" "g4:MMS2UT_GEMM_PP=0 MMS2UT_GEMM_GROUP_M=4" "g2:MMS2UT_GEMM_PP=0 MMS2UT_GEMM_GROUP_M=2" "g16:MMS2UT_GEMM_PP=0 MMS2UT_GEMM_GROUP_M=16" "band:MMS2UT_GEMM_PP=0 MMS2UT_GEMM_GROUP_M=0" "ntst:MMS2UT_GEMM_PP=0 MMS2UT_LIB=$L/libmms2ut_hip_ntst.so" "pp:MMS2UT_GEMM_PP=-1" "ppband:MMS2UT_GEMM_PP=-1 MMS2UT_GEMM_GROUP_M=0" "base2:MMS2UT_GEMM_PP=0" || exit 1
for v in "base:" "band:MMS2UT_GEMM_GROUP_M=0" "ntst:MMS2UT_LIB=$L/libmms2ut_hip_ntst.so"; do
  n=${v%%:*}; e=${v#*:}
  env MMS2UT_GEMM_PP=0 $e timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$n -o run -- python scripts/gemm_l2_ab.py 5 > $O/pmc_fetch_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc_fetch_$n.log; exit 1; }
  env MMS2UT_GEMM_PP=0 $e timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_hit_$n -o run -- python scripts/gemm_l2_ab.py 5 > $O/pmc_hit_$n.log 2>&1 || { echo "pmc hit $n failed"; tail -5 $O/pmc_hit_$n.log; exit 1; }
done
python scripts/pmc_dispatch.py $O/pmc_fetch_base $O/pmc_fetch_band $O/pmc_fetch_ntst $O/pmc_hit_base $O/pmc_hit_band $O/pmc_hit_ntst > $O/pmc_summary.txt 2>&1; tail -40 $O/pmc_summary.txt
