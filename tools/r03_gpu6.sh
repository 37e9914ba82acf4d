#!/bin/bash
# round 3: configs[4] K1 at 512 threads: parity, A/B against the pipelined loop, PMC traffic, bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -v --timeout 300 --timeout-method thread -k "c5_geometry or hybrid" > gpurun_out/r03_t9.log 2>&1 && \
bash tools/ab_c5only.sh base t512p base > gpurun_out/r03_ab_t512p.txt 2>&1 && \
TAG=c5 BENCH_ARGS="--width 16777216 --depth 8" bash tools/pmc_cm.sh && \
timeout -k 10 300 python -u bench.py --width 16777216 --depth 8 > gpurun_out/r03_c5_b6.json 2> gpurun_out/r03_c5_b6.err
