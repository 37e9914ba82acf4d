#!/bin/bash
# rocprofv3 evidence for one Count-Min bench geometry (GPU box):
#   kernel-trace stats, FETCH_SIZE and WRITE_SIZE passes (HBM traffic per dispatch,
#   corrected by tools/pmc_traffic.py), two SQ counter passes.  One pass per run.
# usage: TAG=c5 BENCH_ARGS="--width 16777216 --depth 8" tools/pmc_cm.sh
#   then: tools/pmc_traffic.py gpurun_out/pmc_$TAG/fetch/*counter_collection.csv \
#         gpurun_out/pmc_$TAG/write/*counter_collection.csv profiles/traffic_cm_d8_w16777216_k37_b100000000.json (geometry + device batch)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
T=${TAG:-c2}
O=gpurun_out/pmc_$T
B="python3 bench.py --steps 3 --warmup 1 --no-cpu --windows 0 ${BENCH_ARGS:-}"
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o cm -- $B > $O/trace.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o cm -- $B > $O/fetch.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o cm -- $B > $O/write.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $O/sq1 -o cm -- $B > $O/sq1.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/sq2 -o cm -- $B > $O/sq2.log 2>&1
