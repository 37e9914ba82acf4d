#!/bin/bash
# round-3 closing check of the committed tree: GPU suite, smoke, default bench line
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/chk_pytest_gpu.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/chk_bench.json 2> gpurun_out/chk_bench.err && \
timeout -k 10 300 python bench.py --sketch exact > gpurun_out/chk_exact_bench.json 2> gpurun_out/chk_exact_bench.err
