set -e
# attention bench: current library vs the saved baseline build (lib/libmms2ut_hip_base.so)
for r in 1 2; do
for c in "95 106 0.1" "40 250 0.1" "68 250 0.1 1" "80 150 0.1 1"; do
  echo "new : $(python scripts/attn_bench.py $c 2>/dev/null)"
  echo "base: $(MMS2UT_LIB=multimodal-s2ut_amd/lib/libmms2ut_hip_base.so python scripts/attn_bench.py $c 2>/dev/null)"
done; done
