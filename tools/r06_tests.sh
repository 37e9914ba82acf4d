#!/bin/bash
# Round 6: run some GPU test files (args after the tag), one pytest process.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -5; tail -3 gpurun_out/${TAG}_tests.log; exit $rc
