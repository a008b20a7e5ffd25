#!/bin/bash
# N>1 bench path rehearsed on one GPU: 2 ranks over gloo sharing device 0 (parallel.init_from_env
# maps ranks beyond the visible devices onto them when MMS2UT_DIST_BACKEND=gloo)
export MMS2UT_DIST_BACKEND=gloo
python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 4 --warmup 2 --no-cpu-baseline
