#!/bin/bash
# round 3: non-temporal streams (GNS_NT bits) A/B at both geometries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_bench.sh base nt1 nt3 nt31 nt28 base nt1 nt3 nt31 nt28 > gpurun_out/r03_ab_nt_c2.txt 2>&1 && \
bash tools/ab_c5only.sh base nt28 nt31 base nt28 nt31 > gpurun_out/r03_ab_nt_c5.txt 2>&1
