#!/bin/bash
# Round-4: the whole -m gpu suite, smoke, then tools/r04_bench.sh (bench lines + rocprof).
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/full_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/full_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit 2
bash tools/r04_bench.sh
