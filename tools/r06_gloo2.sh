#!/bin/bash
# Rehearsal of bench.py's N-rank path on the one-GPU box: two ranks over gloo on cuda:0
# (RCCL needs one GPU per rank; the data path is the same).  usage: tools/r06_gloo2.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
GNS_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu \
    > $O/gloo2.json 2> $O/gloo2.err || { echo "FAIL gloo2 rc=$?"; tail -20 $O/gloo2.err; exit 1; }
tail -c 700 $O/gloo2.json
