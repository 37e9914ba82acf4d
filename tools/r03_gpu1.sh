#!/bin/bash
# round 3: configs tests, configs[0] bench, headline bench + its rocprofv3 kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -v --timeout 300 --timeout-method thread -k c1 > gpurun_out/r03_t5.log 2>&1 && \
timeout -k 10 300 python -u bench.py --config c1 > gpurun_out/r03_c1.json 2> gpurun_out/r03_c1.err && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03_b2.json 2> gpurun_out/r03_b2.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b2 -o cm -- python3 bench.py > gpurun_out/r03_b2_prof.json 2> gpurun_out/r03_b2_prof.err
