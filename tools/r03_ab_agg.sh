#!/bin/bash
# round 3: exact P4 table size (2 vs 1 workgroup per CU) and wave folding A/B, then kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_bench_ex.sh base agg6k agg6knf agg3knf base agg6k agg6knf agg3knf > gpurun_out/r03_ab_agg.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ex2 -o ex -- python bench.py --sketch exact --steps 5 --warmup 2 --no-cpu > gpurun_out/prof_ex2.log 2>&1
