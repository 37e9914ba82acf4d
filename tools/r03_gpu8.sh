#!/bin/bash
# round 3: K1 size sums as 32-bit halves: parity (designated-bucket paths, both geometries) and A/B vs the previous K1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_cm_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_t11.log 2>&1 && \
bash tools/ab_c5only.sh prev base prev base > gpurun_out/r03_ab_sum32_c5.txt 2>&1 && \
bash tools/ab_bench.sh prev base c2p5 prev base c2p5 > gpurun_out/r03_ab_sum32_c2.txt 2>&1
