#!/bin/bash
# Round-2 closing evidence run (after the exact sort-word change): the whole chain of
# tools/r02_final.sh plus rocprofv3 kernel stats of the exact-aggregator bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/r02_final.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ex -o ex -- python3 bench.py --sketch exact --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_ex.log 2>&1 || exit 9
ls gpurun_out/prof_cm gpurun_out/prof_ex
