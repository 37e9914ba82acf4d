#!/bin/bash
# Round 6: the whole -m gpu suite (one process), then smoke().
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-r06}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_full_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -4 gpurun_out/${tag}_gpu_full_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/${tag}_smoke.log
