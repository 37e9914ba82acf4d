#!/bin/bash
# round 3: exact aggregator with designated heavy flows: parity tests, then the bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py tests/test_thrift_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r03_exact_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --sketch exact --steps 5 --warmup 2 --no-cpu > gpurun_out/r03_exact_bench.json 2> gpurun_out/r03_exact_bench.err
