#!/bin/bash
# K1 hot-group aggregation / 512-thread C5 K1: A/B at both geometries + parity of the variant
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash tools/ab_c5only.sh base hagg t512 hagg512 base > gpurun_out/r03_ab_hagg_c5.txt 2>&1 && \
bash tools/ab_bench.sh base hagg base hagg > gpurun_out/r03_ab_hagg_c2.txt 2>&1 && \
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_hagg.so timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py tests/test_cm_gpu.py -x -q --timeout 300 --timeout-method thread -k "c5_geometry or designat or hot or insert_keys_parity or headers" > gpurun_out/r03_hagg_tests.log 2>&1
