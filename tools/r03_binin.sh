#!/bin/bash
# round 3: K3s with the bin kept in the staged entry word: Count-Min parity, headline A/B; exact P4 fold A/B by kernel time
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_cm_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py::test_c5_geometry_header_records -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_binin_tests.log 2>&1 && \
bash tools/ab_bench.sh base nobinin base nobinin base nobinin > gpurun_out/r03_ab_binin.txt 2>&1 && \
for v in base fold1; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_$v -o ex -- python bench.py --sketch exact --steps 6 --warmup 2 --no-cpu > gpurun_out/pf_$v.log 2>&1 || exit 1
done
