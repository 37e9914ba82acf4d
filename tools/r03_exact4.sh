#!/bin/bash
# round 3: exact with priority-ordered designation and displaced designated flows folded in X1b: parity + kernel times
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py tests/test_thrift_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_exact4_tests.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_base -o ex -- python bench.py --sketch exact --steps 8 --warmup 2 --no-cpu > gpurun_out/r03_exact4_bench.json 2> gpurun_out/pf_base.log
