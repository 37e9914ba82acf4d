#!/bin/bash
# Bench-only A/B of in-tree library variants (no tests): one JSON line each.
# usage: tools/ab_bench.sh name1 name2 ...   ("base" = go2netspectra_amd/libgns_sketch.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.err
  rc=$?
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_bench_$v.json').read()); print('$v', d['value'], d['stage_ms_per_step'])" | tee -a gpurun_out/ab.log
  if [ $rc -ne 0 ]; then echo "stop rc=$rc"; exit $rc; fi
done
