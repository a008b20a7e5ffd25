#!/bin/bash
# N>1 bench path rehearsed on one GPU: `bench.py --gpus 2` launches its own two ranks
# (torch.distributed.run as a child process); gloo, both ranks sharing device 0
# (parallel.init_from_env maps ranks beyond the visible devices onto them when
# MMS2UT_DIST_BACKEND=gloo).  The gradient bucket size is swept over SURVEY §8e's 8/25/64/128 MB:
# every run must report n_gpus 2, identical ranks, no inconsistent step and the same fp32 master
# checksum (the all-reduced sums do not depend on how the flat gradient is cut into buckets).
# usage: scripts/_dp2_rehearsal.sh OUT_DIR
set -e
out=${1:-gpurun_out/dp2}
mkdir -p "$out"
export MMS2UT_DIST_BACKEND=gloo
for mb in 8 25 64 128; do
  timeout -k 10 300 python -u bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline --no-gemm-timing \
    --bucket-mb $mb > "$out/bucket_$mb.json" 2> "$out/bucket_$mb.err"
  tail -1 "$out/bucket_$mb.json"
done
python - "$out" <<'EOF'
import json, sys
out = sys.argv[1]
lines = {mb: json.loads(open(f"{out}/bucket_{mb}.json").read().strip().splitlines()[-1]) for mb in (8, 25, 64, 128)}
ck = {mb: l["optimizer"]["master_checksum"] for mb, l in lines.items()}
ok = all(l["n_gpus"] == 2 and l["optimizer"]["ranks_identical"] and not l["optimizer"]["inconsistent"]
         for l in lines.values()) and len(set(ck.values())) == 1
print(json.dumps({"n_gpus": {mb: l["n_gpus"] for mb, l in lines.items()}, "master_checksum": ck,
                  "ms_per_step": {mb: l["ms_per_step"] for mb, l in lines.items()}, "ok": ok}))
sys.exit(0 if ok else 1)
EOF
