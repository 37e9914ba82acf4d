#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each) of the SuperSpread bench's kernels.
# usage (GPU box): tools/pmc_ss.sh ; then tools/pmc_traffic.py <fetch csv> <write csv> profiles/traffic_ss_latest.json
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && \
B="python3 bench.py --sketch superspread --steps 2 --warmup 1 --no-cpu" && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_ss_fetch -o ss -- $B > gpurun_out/pmc_ss_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_ss_write -o ss -- $B > gpurun_out/pmc_ss_write.log 2>&1
