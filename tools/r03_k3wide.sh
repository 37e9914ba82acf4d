#!/bin/bash
# round 3: K3s at configs[4] geometry with 1024 threads and one counter buffer (GNS_K3_WIDE): parity + A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
GNS_LIB=$PWD/go2netspectra_amd/libgns_sketch_wide.so timeout -k 10 400 python -u -m pytest tests/test_configs_gpu.py::test_c5_geometry_header_records "tests/test_cm_gpu.py::test_wide_rows_parity" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_wide_tests.log 2>&1 && \
bash tools/ab_c5only.sh base wide base wide > gpurun_out/r03_ab_wide.txt 2>&1
