#!/bin/bash
# round 3: X1 designated-flow wave folding: exact parity, then kernel-time A/B against per-lane atomics
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_exact_gpu.py tests/test_edges_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_exfold_tests.log 2>&1 && \
for v in base nofold; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_$v -o ex -- python bench.py --sketch exact --steps 8 --warmup 2 --no-cpu > gpurun_out/pf_$v.json 2> gpurun_out/pf_$v.log || exit 1
done
