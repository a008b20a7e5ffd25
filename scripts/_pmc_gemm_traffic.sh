#!/bin/bash
# FETCH_SIZE / WRITE_SIZE (separate passes) of isolated GEMMs: scripts/gemm_one.py per shape.
# usage: scripts/_pmc_gemm_traffic.sh "M N K akc bkc [s]" ...
export TMPDIR=/tmp
i=0
for shape in "$@"; do
  i=$((i+1))
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmcg_${i}_$c -o run -- python scripts/gemm_one.py $shape 1 4 > gpurun_out/pmcg_${i}_$c.log 2>&1 || { echo "pmc $shape $c failed"; tail -3 gpurun_out/pmcg_${i}_$c.log; exit 1; }
  done
  python - "$shape" $i <<'PY'
import csv, sys
shape, i = sys.argv[1], sys.argv[2]
def last(c):
    rows = [r for r in csv.DictReader(open(f"gpurun_out/pmcg_{i}_{c}/run_counter_collection.csv")) if "gemm" in r["Kernel_Name"]]
    return float(rows[-1]["Counter_Value"]) * 1024
M, N, K = (int(x) for x in shape.split()[:3])
alg = 2 * (M * K + N * K) + 2 * M * N
f, w = 2 * last("FETCH_SIZE"), last("WRITE_SIZE")
print(f"{shape}: fetch {f/1e6:.1f} MB write {w/1e6:.1f} MB  algorithmic {alg/1e6:.1f} MB  ratio {(f+w)/alg:.2f}")
PY
done
