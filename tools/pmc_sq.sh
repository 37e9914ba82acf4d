#!/bin/bash
# SQ / TCC counter passes over the Count-Min bench (one pass per counter group).
# usage: tools/pmc_sq.sh   (on the GPU box; CSVs under gpurun_out/pmc_*)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
B="python3 bench.py --steps 2 --warmup 1 --no-cpu ${PMC_BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_sq1 -o cm -- $B > gpurun_out/pmc_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc_sq2 -o cm -- $B > gpurun_out/pmc_sq2.log 2>&1
