#!/bin/bash
# round 3: exact aggregator with the hand-written partition + per-bin LDS aggregation: parity, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py tests/test_thrift_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_exact3_tests.log 2>&1 && \
bash tools/ab_bench_ex.sh base base > gpurun_out/r03_exact3_ab.txt 2>&1
