#!/bin/bash
# Round 5: the heavy-hitter list without rocPRIM -- its GPU tests, then its timing
# at the headline geometry (tools/hh_probe.py: 1 and 8 windows of 100M packets).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_cm_gpu.py tests/test_configs_gpu.py tests/test_edges_gpu.py tests/test_growth_gpu.py -m gpu \
  > gpurun_out/r05_hh_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_hh_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/hh_probe.py 1 > gpurun_out/r05_hh_probe1.txt 2>&1 && cat gpurun_out/r05_hh_probe1.txt
