#!/bin/bash
# round 3: exact P4 wave folding (flows folded per wave and chunk) parity + A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py tests/test_configs_gpu.py::test_hybrid_concurrent_exact_and_countmin -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_fold_tests.log 2>&1 && \
bash tools/ab_bench_ex.sh base fold1 fold8 base fold1 fold8 > gpurun_out/r03_ab_fold.txt 2>&1
