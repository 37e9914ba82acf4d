#!/bin/bash
# round 3: exact aggregator, tail words block-compacted in X1: parity, then A/B of the designated-flow count
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py tests/test_thrift_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_exact2_tests.log 2>&1 && \
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_hot10.so timeout -k 10 300 python -u -m pytest tests/test_exact_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_exact2_tests_hot10.log 2>&1 && \
bash tools/ab_bench_ex.sh base hot9 hot10 base hot9 hot10 > gpurun_out/r03_ab_exhot.txt 2>&1
