#!/bin/bash
# Round 5: a subset of the -m gpu suite (files given as arguments after the tag).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/${tag}_gpu_tests.log
exit $rc
