#!/bin/bash
# Bench-only A/B of library variants at the bench geometry and at configs[4]'s (d=8 w=2^24).
# usage: tools/ab_c5.sh name1 name2 ...   ("base" = go2netspectra_amd/libgns_sketch.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  for geo in c2 c5; do
    extra=""; [ $geo = c5 ] && extra="--width 16777216 --depth 8 --steps 3 --warmup 1"
    GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --windows 0 $extra > gpurun_out/ab_${geo}_$v.json 2> gpurun_out/ab_${geo}_$v.err || { echo "stop $v $geo"; tail -5 gpurun_out/ab_${geo}_$v.err; exit 2; }
    python3 -c "import json; d=json.loads(open('gpurun_out/ab_${geo}_$v.json').read().strip().splitlines()[-1]); print('$v $geo', d['value'], d['stage_ms_per_step'])"
  done
done
