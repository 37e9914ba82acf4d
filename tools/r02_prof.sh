#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench path (gloo, both ranks on this GPU), then
# the headline bench under rocprofv3 (kernel stats) and the FETCH/WRITE PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
GNS_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
  > gpurun_out/r02_n2_gloo.json 2> gpurun_out/r02_n2_gloo.err || { tail -20 gpurun_out/r02_n2_gloo.err; exit 3; }
tail -c 400 gpurun_out/r02_n2_gloo.json
tools/pmc_cm.sh || exit 4
ls gpurun_out/prof_cm gpurun_out/pmc_fetch gpurun_out/pmc_write
