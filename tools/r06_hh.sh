#!/bin/bash
# Round 6: the heavy-hitter list at the driver's bench shape (25 + 10 windows of
# 100M packets: 130K / 101K entries), phase-timed (GNS_HH_TRACE), then the HH tests.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-r06_hh}
GNS_HH_TRACE=1 timeout -k 10 300 python -u tools/hh_probe.py 25 10 > gpurun_out/${TAG}_probe.txt 2>&1
rc=$?; echo "probe rc=$rc"; grep -v "^\[hh\]" gpurun_out/${TAG}_probe.txt | tail -12; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_cm_gpu.py tests/test_edges_gpu.py -m gpu > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; exit $rc
