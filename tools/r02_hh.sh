#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/hh_probe.py 60 > gpurun_out/hh_probe.log 2>&1 || { tail gpurun_out/hh_probe.log; exit 2; }
grep -E "hh|C call" gpurun_out/hh_probe.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_hh -o hh -- python3 tools/hh_probe.py 60 > gpurun_out/prof_hh.log 2>&1 || exit 3
python3 tools/prof_summary.py gpurun_out/prof_hh | head -30
