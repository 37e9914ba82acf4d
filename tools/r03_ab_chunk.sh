#!/bin/bash
# round 3: K1/K3s block size (packets per K1 block, GNS_CHUNK) A/B: parity of each variant, then the headline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for v in ch8; do
  GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_$v.so timeout -k 10 300 python -u -m pytest tests/test_cm_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_chunk_tests_$v.log 2>&1 || exit 1
done && \
bash tools/ab_bench.sh base ch32 ch8 base ch32 ch8 > gpurun_out/r03_ab_chunk.txt 2>&1
