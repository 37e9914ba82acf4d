#!/bin/bash
# configs[4] K1 timing ablations (results not exact): where K1's time goes at d=8 w=2^24
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_c5only.sh base hic noidx nohist all3 base > gpurun_out/r03_ab_c5.txt 2>&1
