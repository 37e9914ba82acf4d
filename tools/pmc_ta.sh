#!/bin/bash
# Address-path counters (TA / TCP / GRBM) over the Count-Min bench: is K1 TA- or L1-bound?
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_TA_BUSY TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum --output-format csv -d gpurun_out/pmc_ta1 -o cm -- $B > gpurun_out/pmc_ta1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_DATA_STALLED_BY_TC_CYCLES_sum TA_BUFFER_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_LFIFO_STALL_CYCLES_sum TCP_GATE_EN1_sum --output-format csv -d gpurun_out/pmc_ta2 -o cm -- $B > gpurun_out/pmc_ta2.log 2>&1
