set -e
for r in 1 2; do
for c in "95 106 0.1" "40 250 0.1" "68 250 0.1 1" "80 150 0.1 1" "100 60 0.1 1"; do
  echo "default: $(python scripts/attn_bench.py $c 2>/dev/null)"
  echo "nw4    : $(MMS2UT_ATTN_FWD_NW=4 python scripts/attn_bench.py $c 2>/dev/null)"
done; done
