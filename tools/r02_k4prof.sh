#!/bin/bash
# K4 phase cycles (GNS_K4_PROF build) at the bench geometry and the configs[4] geometry.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
L=$PWD/go2netspectra_amd/libgns_sketch_k4prof.so
GNS_LIB=$L timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 --windows 0 > gpurun_out/k4prof_c2.json 2>&1 || exit 2
GNS_LIB=$L timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 --windows 0 --width 16777216 --depth 8 > gpurun_out/k4prof_c5.json 2>&1 || exit 3
for f in c2 c5; do python3 -c "import json; d=json.loads(open('gpurun_out/k4prof_$f.json').read().strip().splitlines()[-1]); print('$f', d['stage_ms_per_step'], list(d['engine_counters'].values()))"; done
