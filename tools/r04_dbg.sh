#!/bin/bash
# SuperSpread diagnosis: bin sizes and P4 phase ticks per batch (GNS_SS_DEBUG).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/dbg
GNS_SS_DEBUG=1 timeout -k 10 200 python3 bench.py --sketch superspread --no-cpu --steps 3 --warmup 1 > gpurun_out/dbg/ss.json 2> gpurun_out/dbg/ss.err || exit 3
grep gns_ss gpurun_out/dbg/ss.err
