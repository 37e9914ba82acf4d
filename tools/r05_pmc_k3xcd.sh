#!/bin/bash
# HBM traffic of K3s with and without the XCD-contiguous block order (GNS_K3_XCD=1 default / 0):
# FETCH_SIZE and WRITE_SIZE passes of the headline bench, one pass per run.
# then: tools/pmc_traffic.py gpurun_out/<tag>/x<v>_fetch/*counter_collection.csv gpurun_out/<tag>/x<v>_write/*counter_collection.csv out.json
# usage: tools/r05_pmc_k3xcd.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
O=gpurun_out/$1
mkdir -p $O
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --windows 0"
for v in 0 1; do
  export GNS_K3_XCD=$v
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/x${v}_fetch -o cm -- $B > $O/x${v}_fetch.log 2>&1 || { echo "FAIL fetch $v"; tail -5 $O/x${v}_fetch.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/x${v}_write -o cm -- $B > $O/x${v}_write.log 2>&1 || { echo "FAIL write $v"; tail -5 $O/x${v}_write.log; exit 1; }
  echo "xcd=$v done"
done
