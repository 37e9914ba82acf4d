#!/bin/bash
# Round 5: the tests this round added or touched (keyed routing, routed queries,
# GPUTask replay, compact side bounds), each step under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_route_gpu.py tests/test_route_mp_gpu.py tests/test_gputask_replay_gpu.py \
  tests/test_configs_gpu.py -k "not c1 and not pcapgen" > gpurun_out/r05_new_tests.log 2>&1
echo "tests rc=$?"
tail -5 gpurun_out/r05_new_tests.log
