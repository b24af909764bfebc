#!/bin/bash
# Two RCCL ranks of the brick-decomposed bench (small box).  On a one-GPU box both ranks
# share device 0, which RCCL may refuse; on a multi-GPU node this is the N=2 path.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --edge 24 --steps 10 --warmup 2
