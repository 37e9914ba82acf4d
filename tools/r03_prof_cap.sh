#!/bin/bash
# round 3: exact P4 table capacity A/B by kernel time (3072: two workgroups per CU, flush above 2048 flows;
# 3328: two per CU, flush above 2304; 6144: one per CU)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for v in base cap3328 cap6144; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pf_$v -o ex -- python bench.py --sketch exact --steps 8 --warmup 2 --no-cpu > gpurun_out/pf_$v.log 2>&1 || exit 1
done
