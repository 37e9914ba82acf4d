#!/bin/bash
# round 3: packet-major bin codes at d=4 (K1 one 16-byte store, K3s one 16-byte load per sub-pass):
# Count-Min parity (all paths), then headline A/B against the row-major layout
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py tests/test_route_gpu.py tests/test_thrift_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_pmajor_tests.log 2>&1 && \
bash tools/ab_bench.sh base rowmaj base rowmaj base rowmaj > gpurun_out/r03_ab_pmajor.txt 2>&1
