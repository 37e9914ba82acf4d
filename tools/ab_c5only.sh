#!/bin/bash
# Bench-only A/B at configs[4]'s geometry (d=8 w=2^24) of in-tree library variants.
# usage: tools/ab_c5only.sh name1 name2 ...   ("base" = go2netspectra_amd/libgns_sketch.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=go2netspectra_amd/libgns_sketch.so; else lib=go2netspectra_amd/libgns_sketch_$v.so; fi
  GNS_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu --windows 0 --width 16777216 --depth 8 --steps 3 --warmup 1 > gpurun_out/ab_c5_$v.json 2> gpurun_out/ab_c5_$v.err || { echo "stop $v"; tail -5 gpurun_out/ab_c5_$v.err; exit 2; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_c5_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['stage_ms_per_step'])"
done
