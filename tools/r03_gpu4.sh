#!/bin/bash
# round 3: fixed pcapng test, HH beyond 2^26 candidates, headline bench + rocprofv3 stats, C5 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_exact_gpu.py tests/test_cm_gpu.py -v --timeout 300 --timeout-method thread -k "pcapng or 2p26" > gpurun_out/r03_t7.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03_b4.json 2> gpurun_out/r03_b4.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b4 -o cm -- python3 bench.py > gpurun_out/r03_b4_prof.json 2> gpurun_out/r03_b4_prof.err && \
timeout -k 10 300 python -u bench.py --width 16777216 --depth 8 > gpurun_out/r03_c5_b4.json 2> gpurun_out/r03_c5_b4.err
