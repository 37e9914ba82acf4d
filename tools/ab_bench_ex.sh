#!/bin/bash
# Bench-only A/B of library variants on the exact-aggregator bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --sketch exact --steps 3 --warmup 1 --no-cpu > gpurun_out/abx_$v.json 2> gpurun_out/abx_$v.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abx_$v.json').read()); print('$v', d['value'], d['stage_ms_per_step'])"
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; exit $rc; fi
done
