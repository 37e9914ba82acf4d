#!/bin/bash
# round 3: full GPU suite after the parser / frame-decoder change, then the headline bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_t6.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03_b3.json 2> gpurun_out/r03_b3.err
