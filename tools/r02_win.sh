#!/bin/bash
# Headline bench with the per-window exchange (N=1), then the 2-rank gloo rehearsal on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/win_n1.json 2> gpurun_out/win_n1.err || { tail -20 gpurun_out/win_n1.err; exit 2; }
tail -c 900 gpurun_out/win_n1.json
GNS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/win_n2_gloo.json 2> gpurun_out/win_n2_gloo.err || { tail -20 gpurun_out/win_n2_gloo.err; exit 3; }
tail -c 900 gpurun_out/win_n2_gloo.json
