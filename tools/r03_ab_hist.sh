#!/bin/bash
# K1 histogram / designated-bucket summary ablations (timing only, results not exact), both geometries
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_c5only.sh base nohist nohothist nocoldhist nohotsum > gpurun_out/r03_ab_hist_c5.txt 2>&1 && \
bash tools/ab_bench.sh base nohist nohothist nocoldhist nohotsum > gpurun_out/r03_ab_hist_c2.txt 2>&1
