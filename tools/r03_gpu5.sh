#!/bin/bash
# round 3: HH beyond 2^26 candidates, host-input paths (double-buffered staging), headline bench + rocprofv3, C5 bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_exact_gpu.py tests/test_cm_gpu.py -v --timeout 300 --timeout-method thread -k "pcapng or 2p26 or insert_keys_parity or tuples" > gpurun_out/r03_t8.log 2>&1 && \
timeout -k 10 300 python -u bench.py --host-input headers --steps 5 --warmup 1 > gpurun_out/r03_host_h.json 2> gpurun_out/r03_host_h.err && \
timeout -k 10 300 python -u bench.py --host-input tuples --steps 5 --warmup 1 > gpurun_out/r03_host_t.json 2> gpurun_out/r03_host_t.err && \
timeout -k 10 300 python -u bench.py > gpurun_out/r03_b5.json 2> gpurun_out/r03_b5.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b5 -o cm -- python3 bench.py > gpurun_out/r03_b5_prof.json 2> gpurun_out/r03_b5_prof.err && \
timeout -k 10 300 python -u bench.py --width 16777216 --depth 8 > gpurun_out/r03_c5_b5.json 2> gpurun_out/r03_c5_b5.err
