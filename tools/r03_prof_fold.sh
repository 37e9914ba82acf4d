#!/bin/bash
# round 3: P4 fold-count A/B by rocprofv3 kernel time (the bench's stage timers are noisy for P4)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for v in base fold1 fold8; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_$v -o ex -- python bench.py --sketch exact --steps 6 --warmup 2 --no-cpu > gpurun_out/pf_$v.log 2>&1 || exit 1
done
