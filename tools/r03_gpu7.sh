#!/bin/bash
# round 3: K1 summary ablations at 512 threads (C5), C5 bench line with its own PMC traffic, full GPU suite, smoke
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_c5only.sh base no64 nohotsum nocoldhist base > gpurun_out/r03_ab_sum512.txt 2>&1 && \
timeout -k 10 300 python -u bench.py --width 16777216 --depth 8 > gpurun_out/r03_c5_b7.json 2> gpurun_out/r03_c5_b7.err && \
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03_t10.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_smoke.log 2>&1
